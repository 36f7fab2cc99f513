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



def test_fused_norm_decision_modes(monkeypatch):
    """DGI_NORM_FOLD modes: "1" folds on every step of >= the row floor of a routed model (one with
    a GEMM routing table), "table" only where the table prices the fused layer at least as fast,
    "force" on any model, "0" never; steps below the floor never fold."""
    from dgi.models import llama
    from dgi.runtime.gemm_pad import MlpPadTable
    monkeypatch.setattr(llama, "NORM_FOLD_MIN_ROWS", 256)
    grid = [256, 512, 1024]
    raw = [dict(front=1.0, front_mfma=1.0, back=1.0, back_mfma=1.0, pq_blas=1.0, pq_mfma=1.0, po_blas=1.0,
                po_mfma=1.0) for _ in grid]
    raw[2]["front_mfma"] = 2.0                      # at 1,024 rows the all-MFMA layer loses by 1 ms
    t = MlpPadTable.decide(grid, raw, 32)
    rule = lambda rows: t.fold(rows, 1024)          # noqa: E731
    d = llama.fold_decision
    assert d("1", 300, rule) and d("1", 1000, rule) and not d("1", 300, None) and not d("1", 100, rule)
    assert d("table", 300, rule) and not d("table", 1000, rule) and not d("table", 300, None)
    assert d("force", 300, None) and not d("force", 100, None)
    assert not d("0", 300, rule)
