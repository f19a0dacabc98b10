#!/usr/bin/env python3
"""Register and loop report of the production kernels from their gfx950 assembly (CPU only).

Compiles the given sources device-only (`hipcc --offload-arch=gfx950 -O3 -S`), then prints
per kernel: VGPRs / AGPRs, spilled VGPRs / SGPRs, the scratch bytes per lane; and for the
four-wave kernel's ADMM loop (the innermost loop holding the permlane32 hand-offs) the
instruction mix per iteration: LDS reads / writes, fp64 VALU, waits, barriers.

  python tools/isa_report.py [--src solve_wave.hip solve.hip solve_big.hip] [--filter w4]
"""
import argparse
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "python-mpc_amd", "csrc")


def asm_of(src, out):
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "--cuda-device-only", "-S",
           os.path.join(CSRC, src), "-o", out]
    subprocess.run(cmd, check=True, cwd=CSRC, stderr=subprocess.DEVNULL)
    return open(out).read()


def kernels(s):
    for m in re.finditer(r"\.name:\s+(\S+)\n(.*?)\.wavefront_size", s, re.S):
        name, body = m.group(1), m.group(2)

        def g(k):
            r = re.search(r"\." + k + r":\s+(\d+)", body)
            return int(r.group(1)) if r else 0
        yield name, dict(vgpr=g("vgpr_count"), agpr=g("agpr_count"), vspill=g("vgpr_spill_count"),
                         sspill=g("sgpr_spill_count"), scratch=g("private_segment_fixed_size"))


def admm_loop(s, name):
    i = s.index("\n" + name + ":")
    j = s.index(".Lfunc_end", i)
    blocks, cur = {}, None
    for ln in s[i:j].split("\n"):
        if re.match(r"^(\.LBB\d+_\d+|; %bb\.\d+):", ln):
            cur = None
            m = re.search(r"Header=(BB\d+_\d+) Depth=2", ln)
            if "Parent Loop" in ln:
                lab = re.match(r"^\.L(BB\d+_\d+)", ln)
                cur = lab.group(1) if lab else None
            elif m:
                cur = m.group(1)
            continue
        if cur and ln.startswith("\t") and not ln.strip().startswith(";") and not ln.startswith("\t."):
            blocks.setdefault(cur, []).append(ln)
    for seg in blocks.values():
        if sum("permlane32_swap" in x for x in seg) >= 4:
            return seg
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--src", nargs="+", default=["solve_wave.hip"])
    ap.add_argument("--filter", default="")
    a = ap.parse_args()
    with tempfile.TemporaryDirectory() as d:
        for src in a.src:
            s = asm_of(src, os.path.join(d, src + ".s"))
            print(f"== {src}")
            for name, r in kernels(s):
                if a.filter and a.filter not in name:
                    continue
                print(f"{name[:72]:72s} vgpr {r['vgpr']:3d} agpr {r['agpr']:3d} vspill {r['vspill']:3d} "
                      f"sspill {r['sspill']:3d} scratch {r['scratch']:3d} B/lane")
            for name, _ in kernels(s):
                if "k_setup_solve_w4" not in name or "Lb0" not in name or "ILi6ELi4ELi5" not in name:
                    continue
                seg = admm_loop(s, name)
                if seg:
                    c = lambda p: sum(bool(re.search(p, x)) for x in seg)  # noqa: E731
                    print(f"ADMM loop of {name[:40]}...: {len(seg)} instructions per iteration: "
                          f"ds_read {c('ds_read')}, ds_write {c('ds_write')}, fp64 VALU {c('_f64')}, "
                          f"permlane {c('permlane')}, s_waitcnt {c('s_waitcnt')}, s_barrier {c('s_barrier')}, "
                          f"scratch {c('scratch_')}, v_readlane {c('v_readlane')}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
