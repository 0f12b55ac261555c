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


def test_parquet_decoder_under_asan_ubsan(tmp_path):
    """csrc/io/parquet_core.h on pyarrow-written seeds of every covered layout (codec, dictionary,
    page version, nulls, every physical type), then on 20k mutations of them."""
    import itertools

    import numpy as np
    import pyarrow as pa
    import pyarrow.parquet as pq

    rng = np.random.default_rng(0)
    n = 700
    tbl = pa.table({"i32": pa.array(rng.integers(-9, 9, n).astype(np.int32)), "i64": pa.array(rng.integers(0, 5, n)),
                    "f32": pa.array(rng.random(n).astype(np.float32)),
                    "f64": pa.array(rng.random(n), mask=rng.random(n) < 0.2),
                    "b": pa.array(rng.random(n) < 0.5, mask=rng.random(n) < 0.1)})
    seeds = []
    for comp, dic, dpv in itertools.product(["NONE", "SNAPPY"], [False, True], ["1.0", "2.0"]):
        p = tmp_path / f"s_{comp}_{dic}_{dpv}.parquet"
        pq.write_table(tbl, p, compression=comp, use_dictionary=dic, data_page_version=dpv, row_group_size=300)
        seeds.append(str(p))
    exe = str(tmp_path / "parquet_fuzz")
    src = os.path.join(ROOT, "tools", "asan", "parquet_fuzz.cpp")
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
           "-fno-sanitize-recover=all", src, "-o", exe]
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-3000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([exe, "20000", *seeds], stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True,
                       timeout=600, env=env)
    assert r.returncode == 0 and "PARQUET_FUZZ_OK" in r.stdout, r.stdout[-5000:]
