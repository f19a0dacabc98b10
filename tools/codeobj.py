"""Read the gfx950 code objects that ship inside libmpcqp.so (host-only; no GPU needed).

The library's .hip_fatbin section holds one clang offload bundle per translation unit; each is
unbundled with clang-offload-bundler, its AMDGPU metadata printed by llvm-readelf --notes, its
instructions by llvm-objdump.  Used by tests/isa_shape.py (the pinned kernel shapes) and by
bench.py / tools/pmc_summary.py (`kernel_code_hash`: the PMC traffic record names the code it
was measured on).
"""
import hashlib
import os
import re
import subprocess
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"
FIELDS = ("vgpr_count", "agpr_count", "sgpr_count", "vgpr_spill_count", "sgpr_spill_count",
          "private_segment_fixed_size", "group_segment_fixed_size")


def tools_present():
    return all(os.path.exists(os.path.join(LLVM, t)) for t in ("llvm-objcopy", "clang-offload-bundler",
                                                                "llvm-readelf", "llvm-objdump"))


def code_objects(lib, workdir):
    """Paths of the gfx950 code objects inside `lib`."""
    fat = os.path.join(workdir, "fat.bin")
    subprocess.run([os.path.join(LLVM, "llvm-objcopy"), f"--dump-section=.hip_fatbin={fat}", lib, os.devnull],
                   check=True, capture_output=True)
    data = open(fat, "rb").read()
    offs = [m.start() for m in re.finditer(re.escape(MAGIC), data)] + [len(data)]
    out = []
    for i in range(len(offs) - 1):
        b = os.path.join(workdir, f"b{i}.bin")
        co = os.path.join(workdir, f"co{i}.elf")
        with open(b, "wb") as f:
            f.write(data[offs[i]:offs[i + 1]])
        subprocess.run([os.path.join(LLVM, "clang-offload-bundler"), "--unbundle", "--type=o", f"--input={b}",
                        f"--targets={TARGET}", f"--output={co}"], check=True, capture_output=True)
        out.append(co)
    return out


def metadata(co):
    """{kernel name: {field: int}} from the code object's AMDGPU metadata note."""
    txt = subprocess.run([os.path.join(LLVM, "llvm-readelf"), "--notes", co], check=True, capture_output=True,
                         text=True).stdout
    out = {}
    for m in re.finditer(r"\n  - (\.\w+:.*?)(?=\n  - \.|\n  amdhsa\.target|\Z)", txt, re.S):
        body = m.group(1)
        nm = re.search(r"\.name:\s+(\S+)", body)
        if not nm:
            continue
        d = {}
        for f in FIELDS:
            r = re.search(r"\." + f + r":\s+(\d+)", body)
            d[f] = int(r.group(1)) if r else 0
        out[nm.group(1)] = d
    return out


def symbol_range(co, name):
    txt = subprocess.run([os.path.join(LLVM, "llvm-readelf"), "-s", co], check=True, capture_output=True,
                         text=True).stdout
    for ln in txt.splitlines():
        f = ln.split()
        if len(f) >= 8 and f[-1] == name and f[3] == "FUNC":
            a = int(f[1], 16)
            return a, a + int(f[2])
    raise KeyError(name)


def instructions(co, name):
    """(instructions, {label: index}) of kernel `name`."""
    a, b = symbol_range(co, name)
    txt = subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", "--symbolize-operands", f"--start-address={a}",
                          f"--stop-address={b}", co], check=True, capture_output=True, text=True).stdout
    ins, labels = [], {}
    for ln in txt.splitlines():
        m = re.match(r"^[0-9a-f]+ <(L\d+)>:", ln)
        if m:
            labels[m.group(1)] = len(ins)
            continue
        if "//" in ln and ln.startswith("\t"):
            ins.append(ln.split("//")[0].strip())
    return ins, labels


def text_bytes(co):
    """(.text address, .text file offset, file bytes) of a code object."""
    txt = subprocess.run([os.path.join(LLVM, "llvm-readelf"), "-S", "-W", co], check=True, capture_output=True,
                         text=True).stdout
    for ln in txt.splitlines():
        f = ln.split()
        if ".text" in f:
            i = f.index(".text")
            return int(f[i + 2], 16), int(f[i + 3], 16), open(co, "rb").read()
    raise KeyError(".text")


def kernel_code_hash(lib, qualname):
    """sha256 (16 hex digits) over the machine code of every instantiation of kernel `qualname`
    ("mpcqp::k_setup_solve_w4") in `lib`: symbol names and their .text bytes, sorted by name."""
    ns, name = qualname.split("::")
    prefix = f"_ZN{len(ns)}{ns}{len(name)}{name}"
    h = hashlib.sha256()
    found = 0
    with tempfile.TemporaryDirectory() as d:
        for co in code_objects(lib, d):
            txt = subprocess.run([os.path.join(LLVM, "llvm-readelf"), "-s", "-W", co], check=True,
                                 capture_output=True, text=True).stdout
            syms = sorted({(f[-1], int(f[1], 16), int(f[2])) for f in (ln.split() for ln in txt.splitlines())
                           if len(f) >= 8 and f[3] == "FUNC" and f[-1].startswith(prefix)})
            if not syms:
                continue
            addr, off, data = text_bytes(co)
            for sym, a, n in syms:
                h.update(sym.encode())
                h.update(data[off + a - addr: off + a - addr + n])
                found += 1
    if not found:
        raise KeyError(qualname)
    return h.hexdigest()[:16]


def library_path():
    return os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "python-mpc_amd", "osqp_amd",
                        "libmpcqp.so")


if __name__ == "__main__":
    import sys
    print(kernel_code_hash(sys.argv[2] if len(sys.argv) > 2 else library_path(), sys.argv[1]))
