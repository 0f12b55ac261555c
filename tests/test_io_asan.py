"""The IO parsers (csrc/io/io_core.h, shared with the _hopsx_io extension) under AddressSanitizer +
UBSan: tools/asan/io_fuzz.cpp round-trips random tf.train.Examples through TFRecord framing and
fuzzes the TFRecord index, Example decoder and CSV parser with mutated inputs (SURVEY §5.2 —
sanitizer builds of the host C++ layer; the GPU sanitizer is not available on this pool)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_io_parsers_under_asan_ubsan(tmp_path):
    exe = str(tmp_path / "io_fuzz")
    src = os.path.join(ROOT, "tools", "asan", "io_fuzz.cpp")
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-msse4.2",
           "-fsanitize=address,undefined", "-fno-sanitize-recover=all", src, "-o", exe]
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-3000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([exe, "20000"], stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=300,
                       env=env)
    assert r.returncode == 0 and "IO_FUZZ_OK" in r.stdout, r.stdout[-5000:]
