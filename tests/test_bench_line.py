"""bench.py's printed line: the driver keeps only the tail of stdout, so the
headline line must stay compact (< 4 KB) and still carry the contract's keys,
the roofline and the CPU baseline; the full record goes to the detail file."""
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import bench  # noqa: E402

CONTRACT = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
            "vs_baseline", "dtype", "data", "config")


def stub_record():
    """a full N = 1 record of the size the r04 bench printed (22.7 KB), from the committed r04 line"""
    return json.loads((ROOT / "profiles" / "r04_bench.json").read_text())


def test_full_record_is_large():
    assert len(json.dumps(stub_record())) > 16000


def test_compact_line_small_and_complete():
    out = stub_record()
    txt = bench.compact_line(out, "gpurun_out/bench_detail.json")
    assert len(txt) < bench.LINE_LIMIT, len(txt)
    line = json.loads(txt)
    for k in CONTRACT:
        assert k in line, k
    assert line["value"] == float(f"{out['value']:.4g}")
    r = line["roofline"]
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert k in r
    assert r["bound"] in ("hbm", "mfma")
    c = line["cpu_baseline"]
    for k in ("value", "unit", "cores", "kind", "sample"):
        assert c[k] is not None
    assert c["kind"] in ("port", "reference")
    assert set(line["phases"]) >= {"decompose", "ajtai", "fold", "cols", "sum_ms"}
    assert line["side"]["reference_ring"]["value"] > 0
    assert line["step_hbm"]["pmc_frac"] is not None
    assert line["detail"] == "gpurun_out/bench_detail.json"


def test_compact_line_multi_gpu_and_timeout():
    out = stub_record()
    out["n_gpus"] = 8
    out["cpu_baseline"] = None
    out["sharded_fold"] = {"value": 40.0, "unit": "sharded fold-steps/s", "ms_per_step": 25.0, "verified": True,
                           "comm_size": 8, "phases": {"x": "y" * 5000}}
    line = json.loads(bench.compact_line(out, "d.json"))
    assert line["sharded_fold"] == {"value": 40.0, "unit": "sharded fold-steps/s", "ms_per_step": 25.0,
                                    "verified": True, "comm_size": 8}
    assert line["cpu_baseline"] is None
    out["sharded_fold"] = {"error": "timeout after 240 s"}
    txt = bench.compact_line(out, "d.json")
    assert len(txt) < bench.LINE_LIMIT
    assert json.loads(txt)["sharded_fold"]["error"].startswith("timeout")


def test_compact_line_never_exceeds_limit():
    out = stub_record()
    out["config"]["workload_short"] = "w" * 3000  # an oversized field: optional parts are dropped first
    txt = bench.compact_line(out, "d.json")
    line = json.loads(txt)
    assert "value" in line and "roofline" in line and "cpu_baseline" in line


def test_emit_writes_detail(tmp_path, capsys):
    out = stub_record()
    path = tmp_path / "detail.json"
    bench.emit(out, str(path))
    printed = capsys.readouterr().out.strip().splitlines()
    assert len(printed) == 1 and len(printed[0]) < bench.LINE_LIMIT
    full = json.loads(path.read_text())
    assert full["small_shape"]["phases"]["decompose"]["kernel"] == "k_decompose_fused"
    assert json.loads(printed[0])["detail"] == str(path)
    assert full["pmc_files"]["src_hash"] == bench.kernel_source_hash()


def test_stale_pmc_files_are_not_used(tmp_path, monkeypatch):
    """a PMC file collected on other kernel sources is ignored"""
    prof = tmp_path / "profiles"
    prof.mkdir()
    doc = {"config": {"d": 1024, "W": 16384, "kappa": 32}, "src_hash": "000000000000",
           "kernels": {"k_decompose_fused": {"hbm_bytes_per_launch": 1.0, "launches": 1}}}
    (prof / "pmc_traffic_d1024_W16384_k32.json").write_text(json.dumps(doc))
    (tmp_path / "latticeum_amd").symlink_to(ROOT / "latticeum_amd")
    monkeypatch.setattr(bench, "ROOT", tmp_path)
    assert bench.load_traffic(1024, 16384, 32) == {}
    assert "pmc_traffic_d1024_W16384_k32.json" in bench._PMC_STALE
    doc["src_hash"] = bench.kernel_source_hash()
    (prof / "pmc_traffic_d1024_W16384_k32.json").write_text(json.dumps(doc))
    assert bench.load_traffic(1024, 16384, 32)["k_decompose_fused"] == 1.0


def test_round6_line_carries_matrix_and_side_op_counters():
    """the r06 evidence line: each phase row has the matrix-pipe busy column, the
    matrix-core kernels are priced against the dense i8 peak, the side ops carry
    their own PMC figures, and the compact line still fits"""
    full = json.loads((ROOT / "profiles" / "r06_bench_detail.json").read_text())
    line = json.loads(bench.compact_line(full, "d.json"))
    assert line["phases"]["cols"][-1] == "mfma_busy"
    assert len(line["phases"]["ajtai"]) == len(line["phases"]["cols"])
    tops, frac = line["i8_mfma"]["ajtai"]
    assert 0 < frac < 1 and abs(tops / bench.I8_DENSE_TOPS - frac) < 1e-3
    m = full["phases"]["ajtai"]["matrix"]
    # d = 1024, W = 2^14, kappa = 32: 1024 slots x 2560 chunks x 64 products of 32^3
    assert m["i8_macs_per_step"] == 1024 * 2560 * 64 * 32 ** 3
    for k in ("ntt_fwd", "ntt_inv", "poseidon2_w16"):
        assert k in line["side"]["side_ops_pmc"]
    assert len(json.dumps(line)) < bench.LINE_LIMIT


def test_side_ops_pmc_config_is_separate():
    """the side ops' PMC files are keyed by their own config, never mistaken for a step line's"""
    assert bench._pmc_doc("traffic", 1024, 16384, 32, "pmc_traffic_side_ops.json", {"d": 1024}) is None
