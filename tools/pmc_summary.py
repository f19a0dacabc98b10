#!/usr/bin/env python3
"""Reduce one tools/gpu_profile.sh pass (gpurun_out/<tag>/) to per-launch numbers of the
bench line's timed kernel:
  traffic.json -- FETCH_SIZE (x2, the gfx950 note of MI355X_MICROARCH.md) + WRITE_SIZE per
                  launch and per instance, against the algorithmic bytes of SURVEY.md §8d D3
  sq.json      -- the SQ / LDS counters per launch (mean over the launches of the kernel)
  stdout       -- both, plus the kernel-trace mean duration
usage: python tools/pmc_summary.py gpurun_out/<tag>
"""
import csv
import glob
import json
import os
import statistics
import sys


KT_STEPS = 10  # tools/gpu_profile.sh's kt run: --steps 10 unless its args override it (read from kt.log)


def rows(pattern):
    out = []
    for f in glob.glob(pattern):
        out += list(csv.DictReader(open(f)))
    return out


def per_launch(rs, kernel):
    by = {}
    for r in rs:
        if kernel not in r["Kernel_Name"]:
            continue
        by.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    return {k: statistics.mean(v) for k, v in by.items()}, {k: len(v) for k, v in by.items()}


def main():
    d = sys.argv[1]
    line = json.loads([ln for ln in open(os.path.join(d, "bench.json")) if ln.startswith("{")][-1])
    kernel = line["roofline"]["kernel"]
    B = line["config"]["batch_per_gpu"]
    alg = line["roofline"]["bytes_per_solve"]
    res = {"kernel": kernel, "workload": line["config"]["workload"], "batch": B}
    # the code the counters were collected on (bench.py::pmc_traffic compares it with the loaded
    # library's): the package of the run (MPCQP_PKG, else this tree's), its production library
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import codeobj
    pkg = os.environ.get("MPCQP_PKG", os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                   "python-mpc_amd"))
    res["code_sha16"] = codeobj.kernel_code_hash(os.path.join(pkg, "osqp_amd", "libmpcqp.so"), kernel)
    kt = rows(os.path.join(d, "kt", "*kernel_stats.csv"))
    for r in kt:
        if kernel.split("::")[-1] in r["Name"]:
            res["kernel_trace_mean_ms"] = float(r["AverageNs"]) / 1e6
            res["kernel_trace_calls"] = int(r["Calls"])
    # the timed steps' launches: the last `steps` launches of the kernel in the kt run (no
    # identity-dispatch or PCIe legs after the timed region), against the bench line's own
    # in-region HIP-event time
    tr = [r for r in rows(os.path.join(d, "kt", "*kernel_trace.csv")) if kernel.split("::")[-1] in r["Kernel_Name"]]
    if tr:
        tr.sort(key=lambda r: int(r["Start_Timestamp"]))
        steps = KT_STEPS
        ktlog = os.path.join(d, "kt.log")
        if os.path.exists(ktlog):  # the kt run's own bench line says how many steps it timed
            js = [ln for ln in open(ktlog) if ln.startswith("{")]
            if js:
                steps = json.loads(js[-1])["steps"]
        dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in tr[-steps:]]
        res["kernel_trace_timed_launches"] = len(dur)
        res["kernel_trace_timed_mean_ms"] = statistics.mean(dur)
        res["bench_kernel_ms"] = line["roofline"]["kernel_ms"]
        res["timed_mean_over_bench"] = statistics.mean(dur) / line["roofline"]["kernel_ms"]
    f, nf = per_launch(rows(os.path.join(d, "pmc_f", "*counter_collection.csv")), kernel)
    w, nw = per_launch(rows(os.path.join(d, "pmc_w", "*counter_collection.csv")), kernel)
    if "FETCH_SIZE" in f and "WRITE_SIZE" in w:
        fetch, write = 2 * f["FETCH_SIZE"] * 1024, w["WRITE_SIZE"] * 1024
        t = dict(res, fetch_size_kib_raw=f["FETCH_SIZE"], write_size_kib_raw=w["WRITE_SIZE"],
                 launches=[nf["FETCH_SIZE"], nw["WRITE_SIZE"]], fetch_bytes_corrected=fetch, write_bytes=write,
                 bytes_per_launch=fetch + write, bytes_per_instance=(fetch + write) / B,
                 algorithmic_bytes_per_instance=alg, traffic_over_algorithmic=(fetch + write) / B / alg,
                 source=f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes), {kernel}, "
                        f"FETCH_SIZE x2 (gfx950 note), mean over launches")
        json.dump(t, open(os.path.join(d, "traffic.json"), "w"), indent=1)
        print(json.dumps(t, indent=1))
    sq = {}
    for p in ("sq1", "sq2"):
        v, _ = per_launch(rows(os.path.join(d, p, "*counter_collection.csv")), kernel)
        sq.update(v)
    if sq:
        sq = dict(res, **{k: round(v, 1) for k, v in sorted(sq.items())})
        if "SQ_WAVE_CYCLES" in sq:
            wc = sq["SQ_WAVE_CYCLES"]
            for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS",
                      "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_VALU"):
                if k in sq:
                    sq[k + "_frac_of_wave_cycles"] = round(sq[k] / wc, 4)
        if "SQ_LDS_IDX_ACTIVE" in sq and "GRBM_GUI_ACTIVE" in sq:
            # LDS-array busy fraction: SQ_LDS_IDX_ACTIVE (summed over the SEs of all XCCs) over
            # CU-cycles; GRBM_GUI_ACTIVE is summed over the 8 XCCs (rocprofv3 -L: DIMENSION_XCC[0:7]),
            # so one XCC's busy cycles x 256 CUs
            sq["gpu_busy_cycles_per_xcc"] = round(sq["GRBM_GUI_ACTIVE"] / 8, 1)
            sq["lds_util_frac"] = round(sq["SQ_LDS_IDX_ACTIVE"] / (sq["GRBM_GUI_ACTIVE"] / 8 * 256), 4)
        if "SQ_WAVE_CYCLES" in sq:
            sq["note"] = "SQ_WAVE_CYCLES is in quad-cycles (rocprofv3 -L); the *_frac_of_wave_cycles ratios use the raw counters"
        if "SQ_LDS_IDX_ACTIVE" in sq and "SQ_LDS_BANK_CONFLICT" in sq:
            sq["lds_bank_conflict_frac"] = round(sq["SQ_LDS_BANK_CONFLICT"] / max(1.0, sq["SQ_LDS_IDX_ACTIVE"]), 4)
        json.dump(sq, open(os.path.join(d, "sq.json"), "w"), indent=1)
        print(json.dumps(sq, indent=1))


if __name__ == "__main__":
    main()
