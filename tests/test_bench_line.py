"""bench.py's stdout line: whatever the run recorded, the line the driver parses is
one JSON object under bench.LINE_MAX_BYTES that round-trips through json.loads and keeps the headline
keys, the roofline, the CPU baseline and every stage's value."""
import copy
import json

import bench

STAGES = ("frames_c3", "frames_c5", "frames_dbow", "frames_stereo", "frames_orb", "frames_orb_detect",
          "frames_orb_extract", "local_ba", "global_ba", "global_ba_map", "global_ba_loop")


def _cpu(unit):
    return {"value": 1234.56, "unit": unit, "cores": 16, "kind": "port", "value_1thread": 77.7, "thread_scaling": 15.9,
            "host_cpus": 256, "cgroup_cpu_quota": 16, "cpu_model": "X" * 300,
            "node_estimate": {"threads": 256, "value": 1.0, "note": "n" * 400}, "sample": "s" * 1000}


def _maximal_out():
    """A record with every key bench.main writes, every string far longer than a real run's."""
    long = "w" * 2000
    out = {k: long for k in ("metric", "unit", "data", "dtype")}
    out.update({"value": 5573701.2, "n_gpus": 8, "steps": 200, "warmup": 20, "ms_per_step": 0.18372,
                "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
                "config": {"workload": long, "nq": 2000, "nt": 2000, "frames_per_step": 256, "global_batch": 2048,
                           "parallelism": long},
                "roofline": {"kernel": long, "bound": "mfma", "achieved": 2856.6, "peak": 5033.2, "unit": long,
                             "peak_source": long, "frac": 0.5676, "algorithmic_ops_per_launch": 524288000000,
                             "valu_epilogue": {"x": long}, "traffic": 43899674, "traffic_source": long,
                             "kernel_us": 183.5, "kernel_us_backtoback_after_spin": 183.0,
                             "kernel_us_le_ms_per_step": True, "algorithmic_bytes_per_launch": 38912000,
                             "hbm_frac_if_priced_as_hbm": 0.02},
                "single_launch": {"kernel": long, "kernel_us": 5.4, "Mmatches_per_s_kernel": 729413.9, "frac": 0.1,
                                  "note": long},
                "batch_frame0_equals_single": True,
                "roofline_stream": {"kernel": long, "workload": long, "bound": "hbm", "achieved": 6260.2,
                                    "peak": 8000.0, "unit": "GB/s", "frac": 0.78, "traffic": 537046329,
                                    "kernel_us": 85.8, "algorithmic_bytes_per_launch": 1, "Mmatches_per_s": 1.0},
                "stream_train_sharded": {"workload": long, "value": 1.0, "unit": "Mmatches/s", "n_gpus": 8,
                                         "ms_per_step": 1.0, "scaling": "weak", "merged_equal_on_all_ranks": True},
                "cpu_baseline": _cpu("Mmatches/s"), "speedup_vs_cpu": 937.9, "speedup_vs_cpu_1thread": 14718.0,
                "speedup_vs_cpu_node_estimate": 58.62, "detail_file": "gpurun_out/bench_detail.json"})
    for k in STAGES:
        out[k] = {"metric": long, "value": 33571.7, "unit": long, "workload": long, "kernel_frames_per_s": 1.0,
                  "kernel_speedup_vs_cpu": 2.0, "ms_per_call": 3.0, "s_per_gba": 0.1, "peak_device_bytes": 10 ** 9,
                  "single_call_latency": {f"call{i}": {"gpu_us_median": 1.0, "note": long} for i in range(8)},
                  "wall_cpp_adapter": {"note": long, "thread0_stage_s": {"a": 1.0}},
                  "roofline": {"kernel": long, "frac": 0.07226, "kernel_us": 464.46, "traffic": 2132082520,
                               "mfma_busy_frac_pmc": 0.1088, "pmc_source": long},
                  "kernel_ms_per_step": {f"k{i}": 0.1 for i in range(20)},
                  "cpu_baseline": _cpu(long), "speedup_vs_cpu": 19.01, "speedup_vs_cpu_1thread": 295.8,
                  "error": "e" * 500}
    return out


def test_line_fits_and_round_trips():
    out = _maximal_out()
    line = bench.compact_line(out)
    assert len(line.encode()) <= bench.LINE_MAX_BYTES
    assert "\n" not in line
    d = json.loads(line)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "dtype", "config", "roofline",
              "cpu_baseline"):
        assert k in d, k
    assert d["value"] == out["value"] and d["steps"] == 200 and d["warmup"] == 20
    assert d["roofline"]["frac"] == 0.5676 and d["roofline"]["bound"] == "mfma"
    for k in ("achieved", "peak", "traffic", "kernel_us"):
        assert k in d["roofline"], k
    assert d["cpu_baseline"]["cores"] == 16 and d["cpu_baseline"]["kind"] == "port"
    for k in STAGES:
        assert d[k]["value"] == 33571.7, k
    assert d["local_ba"]["roofline"]["frac"] == 0.07226


def test_line_keeps_detail_on_a_real_sized_record():
    """A record of a real run's size keeps the stages' extras (speedups, CPU rates, roofline traffic)."""
    out = _maximal_out()
    for v in out.values():
        if isinstance(v, dict):
            for k in list(v):
                if isinstance(v[k], str):
                    v[k] = v[k][:60]
    for k in ("metric", "unit", "data", "dtype"):
        out[k] = out[k][:40]
    d = json.loads(bench.compact_line(copy.deepcopy(out)))
    assert d["local_ba"]["roofline"]["traffic"] == 2132082520
    assert d["frames_c3"]["cpu"]["cores"] == 16
    assert d["frames_c3"]["kernel_frames_per_s"] == 1.0


def test_line_of_a_failed_stage():
    out = _maximal_out()
    out["local_ba"] = {"error": "RuntimeError: " + "x" * 490}
    d = json.loads(bench.compact_line(out))
    assert d["local_ba"]["error"].startswith("RuntimeError")


def test_batch_plan_tables_match_the_launchers():
    """osg_hamming_top2_batch_plan names the kernel bench.py prices: its shape tables in
    csrc/hamming_mfma.hip (mfma_shape_of) mirror the launch switches of the I8 and the FP4 forms."""
    import os
    import re
    src = open(os.path.join(os.path.dirname(bench.__file__), "orb_slam3_comments_ghr_amd", "csrc",
                            "hamming_mfma.hip")).read()
    body = src[src.index("int osg_launch_top2_batch_mfma"):]
    split = body.index("\n    switch (shape)")  # the I8 switch; the FP4 one is nested under if (mfma_fp4())
    fp4_sw, i8_sw = body[body.index("if (mfma_fp4())"):split], body[split:]

    def switch(text, fn):
        cases = {int(k): tuple(int(x) for x in v.split(","))
                 for k, v in re.findall(r"case (\d+): return " + fn + r"<(\d+, \d+, \d+, \d+)>", text)}
        cases[0] = tuple(int(x) for x in re.search(r"default: return " + fn + r"<(\d+, \d+, \d+, \d+)>",
                                                   text).group(1).split(","))
        return cases

    def table(name, n):
        t = re.search(r"static const int " + name + r"\[" + str(n) + r"\]\[4\] = \{(.*?)\};", src, re.S).group(1)
        return [tuple(int(x) for x in row.split(",")) for row in re.findall(r"\{([^{}]*)\}", t)]

    i8, f4 = table("i8", 5), table("f4", 14)
    for k, v in switch(i8_sw, "launch").items():
        assert i8[k] == v, (k, v)
    for k, v in switch(fp4_sw, "launch_fp4").items():
        assert f4[k] == v, (k, v)
