"""CPU checks: native IO library (TFRecord framing, tf.train.Example codec, CSV parser, row
gather), fused-optimizer CPU paths vs torch.optim, tensorboard event files, model registry
(export / get_best_model), serving (Python Predict script + torch predictor + inference log)."""
import json
import struct
from pathlib import Path

import numpy as np
import pytest
import torch


# ------------------------------------------------------------------ IO
def test_crc32c_known_vectors():
    from hops_examples_amd import io

    assert io.crc32c(b"123456789") == 0xE3069283  # RFC 3720 check value
    assert io.crc32c(b"") == 0


def test_tfrecord_roundtrip_and_framing(tmp_path):
    from hops_examples_amd import io

    recs = [b"", b"a", bytes(range(256)) * 40]
    p = tmp_path / "x.tfrecord"
    with io.TFRecordWriter(str(p)) as w:
        for r in recs:
            w.write(r)
    assert io.read_tfrecords(str(p)) == recs
    raw = p.read_bytes()
    n = struct.unpack("<Q", raw[:8])[0]
    assert n == 0 and struct.unpack("<I", raw[8:12])[0] == io.masked_crc32c(raw[:8])
    bad = bytearray(raw)
    bad[-5] ^= 0xFF  # corrupt the payload of the last record
    p.write_bytes(bytes(bad))
    with pytest.raises(Exception):
        io.read_tfrecords(str(p), verify=True)


def test_example_codec_and_columnar_decode():
    from hops_examples_amd import io

    ex = io.encode_example({"image": np.arange(6, dtype=np.float32), "label": 7, "name": b"seven"})
    d = io.decode_example(ex)
    np.testing.assert_array_equal(np.asarray(d["image"], np.float32), np.arange(6, dtype=np.float32))
    assert list(d["label"]) == [7] and list(d["name"]) == [b"seven"]
    recs = [io.encode_example({"x": np.full(3, i, np.float32), "y": i}) for i in range(50)]
    cols = io.decode_batch(recs, [("x", "float", 3), ("y", "int64", 1)])
    assert cols["x"].shape == (50, 3) and cols["y"][:, 0].tolist() == list(range(50))


def test_csv_numeric_and_gather(tmp_path):
    from hops_examples_amd import io

    p = tmp_path / "d.csv"
    p.write_text("a,b,c\n1,2.5,x\n3,,4\n")
    names, arr = io.read_csv_numeric(str(p))
    assert names == ["a", "b", "c"]
    assert arr[0, 1] == 2.5 and np.isnan(arr[1, 1]) and np.isnan(arr[0, 2])
    src = np.arange(40, dtype=np.float32).reshape(10, 4)
    dst = np.zeros((3, 4), np.float32)
    io.gather_rows(src, np.array([9, 0, 4]), dst)
    np.testing.assert_array_equal(dst, src[[9, 0, 4]])


# ------------------------------------------------------------------ optimizers
@pytest.mark.parametrize("name,ours,theirs", [
    ("sgd", dict(lr=0.1, momentum=0.5), lambda p: torch.optim.SGD(p, lr=0.1, momentum=0.5)),
    ("adam", dict(lr=0.01), lambda p: torch.optim.Adam(p, lr=0.01, eps=1e-8)),
    ("adamw", dict(lr=0.01, weight_decay=0.1), lambda p: torch.optim.AdamW(p, lr=0.01, weight_decay=0.1)),
    ("adadelta", dict(lr=1.0, rho=0.95, eps=1e-7), lambda p: torch.optim.Adadelta(p, lr=1.0, rho=0.95, eps=1e-7)),
    ("rmsprop", dict(lr=0.01, alpha=0.9, eps=1e-7),
     lambda p: torch.optim.RMSprop(p, lr=0.01, alpha=0.9, eps=1e-7)),
    ("adagrad", dict(lr=0.1, eps=1e-10), lambda p: torch.optim.Adagrad(p, lr=0.1, eps=1e-10)),
])
def test_optimizer_cpu_matches_torch(name, ours, theirs):
    from hops_examples_amd import optim
    from hops_examples_amd.runtime.arena import ParamArena

    torch.manual_seed(0)
    a = torch.nn.Linear(5, 3)
    b = torch.nn.Linear(5, 3)
    b.load_state_dict(a.state_dict())
    ParamArena.from_module(a)
    oa = optim.get(name, a, **ours)
    ob = theirs(b.parameters())
    for i in range(6):
        x = torch.randn(8, 5)
        for m in (a, b):
            m.zero_grad(set_to_none=False) if m is b else None
            (m(x) ** 2).mean().backward()
        oa.step()
        ob.step()
        ob.zero_grad()
    torch.testing.assert_close(a.weight, b.weight, atol=1e-5, rtol=1e-4)
    torch.testing.assert_close(a.bias, b.bias, atol=1e-5, rtol=1e-4)


# ------------------------------------------------------------------ tensorboard / registry / serving
def test_tensorboard_event_file_roundtrip(tmp_path):
    from hops_examples_amd import tensorboard as tb

    w = tb.SummaryWriter(str(tmp_path))
    for s in range(5):
        w.add_scalar("loss", 1.0 / (s + 1), s)
    w.add_histogram("w", np.random.randn(100), 0)
    w.close()
    sc = tb.read_scalars(str(tmp_path))
    assert [round(v, 4) for _, v in sc["loss"]] == [1.0, 0.5, 0.3333, 0.25, 0.2]
    assert next(tmp_path.glob("events.out.tfevents.*")).stat().st_size > 0


def test_model_registry_best_model(project_root, capsys):
    from hops_examples_amd import model

    for acc in (0.9, 0.97, 0.95):
        d = project_root / "tmp_model"
        d.mkdir(parents=True, exist_ok=True)
        (d / "weights.bin").write_bytes(b"w" * 10)
        model.export(str(d), "mnist", metrics={"accuracy": acc})
    out = capsys.readouterr().out
    assert "Exported model mnist as version 3 successfully." in out
    best = model.get_best_model("mnist", "accuracy", model.Metric.MAX)
    assert best["version"] == 2 and best["metrics"]["accuracy"] == "0.97"  # string-valued, as the reference
    assert model.get_best_model("mnist", "accuracy", model.Metric.MIN)["version"] == 1


def test_serving_python_predictor_and_inference_log(project_root):
    from hops_examples_amd import kafka, model, serving

    d = project_root / "iris_model"
    d.mkdir(parents=True)
    (d / "iris_flower_classifier.py").write_text(
        "class Predict:\n"
        "    def __init__(self):\n        self.w = [1, -1, 0.5, 2]\n"
        "    def predict(self, inputs):\n"
        "        return [int(sum(a * b for a, b in zip(self.w, x)) > 0) for x in inputs]\n"
        "    classify = predict\n    regress = predict\n")
    path = model.export(str(d), "IrisFlowerClassifier", metrics={"accuracy": 0.98})
    serving.create_or_update("irisflowerclassifier", path, model_version=1, model_server="FLASK")
    serving.start("irisflowerclassifier")
    try:
        assert serving.get_status("irisflowerclassifier") == "Running"
        r = serving.make_inference_request("irisflowerclassifier", {"inputs": [[1, 0, 0, 0], [0, 1, 0, 0]]})
        assert r["predictions"] == [1, 0]
        topic = serving.get_kafka_topic("irisflowerclassifier")
        c = kafka.Consumer({"group.id": "t", "auto.offset.reset": "earliest"})
        c.subscribe([topic])
        msg = c.poll(timeout=5.0)
        assert msg is not None
        rec = json.loads(msg.value())
        assert rec["modelName"] == "irisflowerclassifier" and "inferenceRequest" in rec
    finally:
        serving.stop("irisflowerclassifier")
    assert serving.get_status("irisflowerclassifier") == "Stopped"


def test_make_step_falls_back_when_the_persistent_grid_cannot_be_resident(monkeypatch):
    """runtime.persist.launchable refuses a device with fewer CUs than the persistent grid (a partitioned
    GPU) or an occupancy below one workgroup per CU, and make_step then builds a TrainStep."""
    from hops_examples_amd.runtime import persist

    monkeypatch.setattr(persist, "geometry", lambda: {"grid": 201, "max_ranks": 8})
    monkeypatch.setattr(persist, "_occupancy", lambda dp: 1)
    monkeypatch.setattr(persist, "_device_cus", lambda dev: 256)
    assert persist.launchable("cuda:0") == (True, "ok")
    monkeypatch.setattr(persist, "_device_cus", lambda dev: 128)  # e.g. a CPX-partitioned MI355X
    ok, why = persist.launchable("cuda:0")
    assert not ok and "128 CUs" in why
    monkeypatch.setattr(persist, "_device_cus", lambda dev: 256)
    monkeypatch.setattr(persist, "_occupancy", lambda dp: 0)
    assert not persist.launchable("cuda:0")[0]


def test_flagship_structure_match_and_make_step_cpu():
    """The persistent engine is chosen by layer structure; on the CPU (no GPU arena) make_step builds a
    TrainStep that trains."""
    import torch

    from hops_examples_amd import optim
    from hops_examples_amd.models.mnist import KerasMnistCNN, MirroredMnistCNN
    from hops_examples_amd.runtime import persist
    from hops_examples_amd.runtime.arena import ParamArena
    from hops_examples_amd.runtime.step import TrainStep, make_step

    m = MirroredMnistCNN()
    assert persist.flagship_layers(m) is not None
    assert persist.flagship_layers(KerasMnistCNN(kernel=2, pool=2)) is None  # different structure (conv k, fc1)

    class Sub(MirroredMnistCNN):  # same layers, same forward: still the flagship
        pass

    assert persist.flagship_layers(Sub()) is not None
    ParamArena.from_module(m, "cpu")
    opt = optim.Adadelta(m, lr=1.0)
    st = make_step(m, opt, "sparse_ce", batch=32)
    assert isinstance(st, TrainStep) and st.kind == "trainstep"
    x = torch.randint(0, 256, (32, 28, 28, 1), dtype=torch.uint8)
    y = torch.randint(0, 10, (32,))
    r = st(x, y)
    assert float(r["loss"].reshape(-1)[0]) > 0
