#!/usr/bin/env python3
"""Turn rocprofv3 PMC passes into profiles/traffic_<workload>_b<B>.json for bench.py.

  rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_f -o f --output-format csv -- python3 bench.py --no-cpu --steps 2
  rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_w -o w --output-format csv -- python3 bench.py --no-cpu --steps 2
  python tools/pmc_traffic.py gpurun_out/pmc_f/f_counter_collection.csv gpurun_out/pmc_w/w_counter_collection.csv \\
      --workload vanilla-lateral-N20 --batch 1024

FETCH_SIZE / WRITE_SIZE are in KiB per dispatch (separate passes: they do not fit
one TCC pass on gfx950).  Per MI355X_MICROARCH.md (HBM section) FETCH_SIZE counts
64 B per 128-B request for wide streaming reads, so it is doubled; WRITE_SIZE is
taken as is.  Both include Infinity-Cache hits.
"""
import argparse
import csv
import json
import os
import statistics


def per_launch(path, kernel_prefix, counter):
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(path))
            if r["Counter_Name"] == counter and kernel_prefix in r["Kernel_Name"]]
    if not vals:
        raise SystemExit(f"no {counter} rows for {kernel_prefix} in {path}")
    return statistics.mean(vals), len(vals)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_csv")
    ap.add_argument("write_csv")
    ap.add_argument("--workload", required=True)
    ap.add_argument("--batch", type=int, required=True)
    ap.add_argument("--kernel", default="mpcqp::k_solve")
    ap.add_argument("--bytes-per-unit", type=float, default=None, help="algorithmic bytes per instance")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    f_kib, nf = per_launch(a.fetch_csv, a.kernel, "FETCH_SIZE")
    w_kib, nw = per_launch(a.write_csv, a.kernel, "WRITE_SIZE")
    fetch = 2 * f_kib * 1024
    write = w_kib * 1024
    res = {"kernel": a.kernel, "workload": a.workload, "batch": a.batch,
           "fetch_size_kib_raw": f_kib, "write_size_kib_raw": w_kib, "launches": [nf, nw],
           "fetch_bytes_corrected": fetch, "write_bytes": write,
           "bytes_per_launch": fetch + write, "bytes_per_instance": (fetch + write) / a.batch,
           "source": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes), {a.kernel}, "
                     f"FETCH_SIZE x2 (gfx950 note), mean over launches"}
    if a.bytes_per_unit:
        res["algorithmic_bytes_per_instance"] = a.bytes_per_unit
        res["traffic_over_algorithmic"] = res["bytes_per_instance"] / a.bytes_per_unit
    out = a.out or os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles",
                                f"traffic_{a.workload}_b{a.batch}.json")
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
