"""Code-object shape of the production library's hot kernels (test helper, CPU only): what
actually ships, read by tools/codeobj.py from libmpcqp.so's bundled gfx950 code objects."""
import os
import re
import subprocess
import sys
import tempfile

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
from codeobj import LLVM, code_objects, instructions, metadata, tools_present  # noqa: E402,F401

def loops(ins, labels):
    """Backward branches: (start, end) instruction index ranges, innermost first by length."""
    out = []
    for i, s in enumerate(ins):
        m = re.match(r"(s_cbranch_\w+|s_branch)\s+(L\d+)", s)
        if m and m.group(2) in labels and labels[m.group(2)] <= i:
            out.append((labels[m.group(2)], i))
    return sorted(out, key=lambda r: r[1] - r[0])


def count(ins, lo, hi, pat):
    return sum(1 for x in ins[lo:hi + 1] if x.startswith(pat))


def census(ins, lo, hi):
    return dict(instructions=hi - lo + 1, barriers=count(ins, lo, hi, "s_barrier"),
                readlane=count(ins, lo, hi, "v_readlane"),
                scratch=count(ins, lo, hi, "scratch_") + count(ins, lo, hi, "buffer_store") +
                count(ins, lo, hi, "buffer_load"))


def report(lib, kernels):
    """{key: metadata + loop census} for kernels = {key: (symbol substring, form)}.  form "w4":
    the four-wave kernel's ADMM loop is the shortest call-free loop with four workgroup barriers
    (rhs, phase B, phase C, rows); form "big": k_solve_b's ADMM loop is the longest call-free
    loop, and its sweep-step loops are the loops nested in it that carry three or more
    barriers and no call."""
    with tempfile.TemporaryDirectory() as d:
        cos = code_objects(lib, d)
        out = {}
        for key, (sub, form) in kernels.items():
            for co in cos:
                md = metadata(co)
                hit = [k for k in md if sub in k]
                if not hit:
                    continue
                name = hit[0]
                r = dict(md[name], symbol=name)
                ins, labels = instructions(co, name)
                free = [(lo, hi) for lo, hi in loops(ins, labels) if count(ins, lo, hi, "s_swappc") == 0]
                if form == "w4":
                    lo, hi = min((t for t in free if count(ins, t[0], t[1], "s_barrier") == 4),
                                 key=lambda t: t[1] - t[0])
                    r["loop"] = census(ins, lo, hi)
                else:
                    lo, hi = max(free, key=lambda t: t[1] - t[0])
                    r["loop"] = census(ins, lo, hi)
                    # the sweep's step loops: the innermost loops of three or more barriers inside
                    # it (each a run of unrolled two-sided sweep steps with a runtime count)
                    bl = [(a, b) for a, b in free if lo <= a and b <= hi and (a, b) != (lo, hi)
                          and count(ins, a, b, "s_barrier") >= 3]
                    inner = [(a, b) for a, b in bl if not any(a <= c and d <= b and (c, d) != (a, b) for c, d in bl)]
                    steps = [census(ins, a, b) for a, b in inner]
                    r["step_loops"] = len(steps)
                    r["step_instructions"] = sum(c["instructions"] for c in steps)
                    r["step_readlane"] = sum(c["readlane"] for c in steps)
                    r["step_scratch"] = sum(c["scratch"] for c in steps)
                out[key] = r
                break
        return out


HOT = {
    # configs[1] (the headline): the fused setup + solve four-wave kernel
    "cfg2": ("_ZN5mpcqp16k_setup_solve_w4ILi6ELi4ELi5ELi6ELi2ELb0ELi6ELb0ELb0ELi0EE", "w4"),
    # configs[2] / [3]: the slack layouts' eliminated-column instantiation
    "cfg3": ("_ZN5mpcqp16k_setup_solve_w4ILi6ELi4ELi8ELi8ELi3ELb1ELi8ELb0ELb0ELi0EE", "w4"),
    # configs[4]: the long-horizon two-sided kernel, variant 12
    "cfg5": ("_ZN5mpcqp9k_solve_bILi512ELi9ELi8ELi2ELi2ELb0ELb0EE", "big"),
    # ... and its persistent form (the batch path: the instance body inlined into the work loop)
    "cfg5p": ("_ZN5mpcqp9k_solve_bILi512ELi9ELi8ELi2ELi2ELb0ELb1EE", "big"),
}

if __name__ == "__main__":
    import json
    import sys
    lib = sys.argv[1] if len(sys.argv) > 1 else os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(
        __file__))), "python-mpc_amd", "osqp_amd", "libmpcqp.so")
    print(json.dumps(report(lib, HOT), indent=1))
