"""Host-side measurement plumbing: PMC traffic table parsing and the bench's lookup of it."""
import csv
import importlib.util
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _load(name, path):
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_kernel_name_shortening_matches_bench_names():
    T = _load("pmc_traffic", os.path.join(ROOT, "tools", "pmc_traffic.py"))
    assert T.short("void (anonymous namespace)::gemm_ring_kernel<128, 128, 2, 2, 4, 1, true, true>(GemmP)") \
        == "gemm_ring_kernel<128, 128, 2, 2, 4, 1, true, true>"
    assert T.short("(anonymous namespace)::ce_row_kernel(unsigned short const*, long)") == "ce_row_kernel"


def test_traffic_table_from_counter_csvs(tmp_path):
    T = _load("pmc_traffic", os.path.join(ROOT, "tools", "pmc_traffic.py"))
    name = "void (anonymous namespace)::gemm_pp3_kernel<4, false, true, 0>(GemmP)"
    # third pass: MFMA busy cycles + GRBM_GUI_ACTIVE in one directory, 10 us dispatches
    passes = (("FETCH_SIZE", "FETCH_SIZE", [100.0, 300.0]), ("WRITE_SIZE", "WRITE_SIZE", [50.0, 50.0]),
              ("SQ_VALU_MFMA_BUSY_CYCLES", "SQ_VALU_MFMA_BUSY_CYCLES", [1024 * 8000.0, 1024 * 8000.0]),
              ("SQ_VALU_MFMA_BUSY_CYCLES", "GRBM_GUI_ACTIVE", [8 * 20000.0, 8 * 20000.0]))
    for wl in ("lm", "qf"):
        for i, (dname, ctr, vals) in enumerate(passes):
            d = tmp_path / f"{wl}_{dname}" / f"host{i}"
            d.mkdir(parents=True)
            with open(d / "run_counter_collection.csv", "w", newline="") as f:
                w = csv.DictWriter(f, fieldnames=["Kernel_Name", "Counter_Name", "Counter_Value",
                                                  "Start_Timestamp", "End_Timestamp"])
                w.writeheader()
                for v in vals:
                    w.writerow(dict(Kernel_Name=name, Counter_Name=ctr, Counter_Value=v,
                                    Start_Timestamp=1000, End_Timestamp=11000))
    import contextlib
    import io
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        T.main(str(tmp_path))
    out = json.loads(buf.getvalue())
    k = out["workloads"]["lm"]["gemm_pp3_kernel<4, false, true, 0>"]
    # FETCH_SIZE doubled (gfx950 streaming-read correction), both counters in KiB
    assert k["launches"] == 2 and k["hbm_bytes"] == round(2 * 200.0 * 1024 + 50.0 * 1024)
    # 8000 busy cycles per SIMD over 20000 cycles per XCD; 20000 cycles in 10 us = 2 GHz
    assert k["mfma_busy"] == 0.4 and k["clock_ghz"] == 2.0


def test_committed_traffic_covers_bench_dominant_kernels():
    with open(os.path.join(ROOT, "profiles", "pmc_traffic.json")) as f:
        t = json.load(f)["workloads"]
    # the dominant GEMMs of the latest committed closing bench line (profiles/r5/bench_r5fin.json:
    # the LM line's and the Q-Former line's roofline kernels), with MFMA busy and the exact
    # MFMA-rate fraction
    with open(os.path.join(ROOT, "profiles", "r5", "bench_r5fin.json")) as f:
        b = json.load(f)
    for wl, name in (("lm", b["roofline"]["kernel"]), ("qf", b["caption_qformer"]["roofline"]["kernel"])):
        assert t[wl][name]["hbm_bytes"] > 0 and 0 < t[wl][name]["mfma_rate_frac"] < 1
