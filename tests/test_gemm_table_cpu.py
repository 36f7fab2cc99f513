"""The shipped GEMM routing table (dgi/tuned/) is only reused on the device it was
measured on: its JSON carries the GPU architecture and HIP release next
to the shape key, and ``load_tuned`` refuses a table whose tag differs."""
import glob
import json
import os

from dgi.runtime import gemm_pad


def test_shipped_table_is_tagged_for_mi355x():
    paths = glob.glob(os.path.join(gemm_pad.TUNED_DIR, "gemm_table_*.json"))
    assert paths
    for p in paths:
        d = json.load(open(p))
        assert d["device"]["arch"] == "gfx950" and d["device"]["hip"]
        assert gemm_pad.tuned_path(d["key"]) == p          # the file name still hashes the key only


def test_load_tuned_refuses_another_device(tmp_path, monkeypatch):
    src = glob.glob(os.path.join(gemm_pad.TUNED_DIR, "gemm_table_*.json"))[0]
    d = json.load(open(src))
    monkeypatch.setattr(gemm_pad, "TUNED_DIR", str(tmp_path))
    here = gemm_pad.device_tag()
    m_max = d["grid"][-1]
    for tag, ok in ((here, True), ({**here, "arch": "gfx942"}, False), ({**here, "hip": "6.1"}, False),
                    (None, False)):
        dd = dict(d)
        if tag is None:
            dd.pop("device")
        else:
            dd["device"] = tag
        with open(gemm_pad.tuned_path(d["key"]), "w") as f:
            json.dump(dd, f)
        t = gemm_pad.load_tuned(d["key"], m_max)
        assert (t is not None) == ok, tag
