"""Register and scratch budget of the gfx950 kernels inside a built libipmc.so,
and the instruction sequence of their RK4 loops.

  python tools/code_objects.py [path/to/libipmc.so] [name substring ...]

The shared library's .hip_fatbin section holds one clang offload bundle per
translation unit; each bundle's gfx950 code object carries the AMDGPU
metadata note (NT_AMDGPU_METADATA) with every kernel's .vgpr_count,
.agpr_count, .vgpr_spill_count and .private_segment_fixed_size (scratch bytes
per lane).  kernels() returns them by kernel name; tests/test_code_objects_cpu.py
holds the headline kernels to the register budget their occupancy target
needs.  Needs only the ROCm LLVM tools (no GPU).
"""
import os
import subprocess
import sys
import tempfile

import yaml

LLVM = "/opt/rocm/lib/llvm/bin"
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(REPO, "ip_mcmc_amd", "lib", "libipmc.so")
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"


def _metadata(code_object):
    """The AMDGPU metadata note of one code object, parsed (YAML)."""
    out = subprocess.run([os.path.join(LLVM, "llvm-readelf"), "--notes", code_object], check=True,
                         capture_output=True, text=True).stdout
    doc = out[out.index("---"):]
    end = doc.find("\n...")
    return yaml.safe_load(doc[:end] if end >= 0 else doc)


def kernels(lib=LIB):
    """{kernel name: metadata dict} over every gfx950 code object in `lib`."""
    with tempfile.TemporaryDirectory() as tmp:
        out = {}
        for co in _code_objects(lib, tmp):
            for k in _metadata(co)["amdhsa.kernels"]:
                out[k[".name"]] = k
        return out


def _code_objects(lib, tmp):
    """Paths of the gfx950 code objects of `lib`'s offload bundles, unbundled into tmp."""
    fat = os.path.join(tmp, "fatbin")
    subprocess.run([os.path.join(LLVM, "llvm-objcopy"), "--dump-section", f".hip_fatbin={fat}", lib,
                    os.path.join(tmp, "discard")], check=True, capture_output=True)
    blob = open(fat, "rb").read()
    starts = []
    i = blob.find(MAGIC)
    while i >= 0:
        starts.append(i)
        i = blob.find(MAGIC, i + 1)
    if not starts:
        raise RuntimeError(f"no offload bundle in {lib}'s .hip_fatbin")
    cos = []
    for n, (a, b) in enumerate(zip(starts, starts[1:] + [len(blob)])):
        bundle = os.path.join(tmp, f"b{n}")
        with open(bundle, "wb") as f:
            f.write(blob[a:b])
        co = os.path.join(tmp, f"b{n}.co")
        subprocess.run([os.path.join(LLVM, "clang-offload-bundler"), "--unbundle", "--type=o", f"--input={bundle}",
                        f"--targets={TARGET}", f"--output={co}"], check=True, capture_output=True)
        cos.append(co)
    return cos


def disassemble(symbol, lib=LIB):
    """[(address, instruction text)] of one kernel of `lib` (llvm-objdump)."""
    import re

    with tempfile.TemporaryDirectory() as tmp:
        for co in _code_objects(lib, tmp):
            out = subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", "--mcpu=gfx950",
                                  f"--disassemble-symbols={symbol}", co], check=True, capture_output=True,
                                 text=True).stdout
            ins = []
            for line in out.split("\n"):
                m = re.match(r"\t(\S.*?)\s*// ([0-9A-F]+):", line)
                if m:
                    tgt = re.search(r"<" + re.escape(symbol) + r"\+0x([0-9a-f]+)>", line)
                    ins.append((int(m.group(2), 16), m.group(1), tgt and int(tgt.group(1), 16)))
            if ins:
                base = ins[0][0]
                return [(a - base, t, off) for a, t, off in ins]
    raise KeyError(f"{symbol} not in {lib}")


def inner_loops(ins):
    """The backward-branch loops of a disassembled kernel, innermost first:
    lists of instruction texts from the branch target to the branch."""
    loops = []
    addr = [a for a, _, _ in ins]
    for i, (a, t, off) in enumerate(ins):
        if off is not None and off <= a and t.startswith(("s_cbranch", "s_branch")):
            j = addr.index(off) if off in addr else None
            if j is not None:
                loops.append([x for _, x, _ in ins[j : i + 1]])
    return sorted(loops, key=len)


def rk_loop(symbol, lib=LIB, dpp=24):
    """The RK4 time loop of a Lorenz-96 sweep kernel: its innermost loop with
    the `dpp` halo moves of one RK4 step (24: three halo values of two dwords
    in four stages)."""
    for body in inner_loops(disassemble(symbol, lib)):
        if sum(x.startswith("v_mov_b32_dpp") for x in body) == dpp:
            return body
    raise KeyError(f"no loop with {dpp} DPP moves in {symbol}")


def fingerprint(body):
    """sha1 of a loop's instructions with their register numbering: what the
    one-wave packed fp32 kernel's speed depends on."""
    import hashlib

    return hashlib.sha1("\n".join(" ".join(x.split()) for x in body).encode()).hexdigest()[:16]


def budget(meta):
    """(VGPRs + AGPRs, scratch bytes per lane, VGPR spills, SGPR spills) of one kernel."""
    return (meta[".vgpr_count"] + meta.get(".agpr_count", 0), meta[".private_segment_fixed_size"],
            meta.get(".vgpr_spill_count", 0), meta.get(".sgpr_spill_count", 0))


def main():
    lib = sys.argv[1] if len(sys.argv) > 1 and sys.argv[1].endswith(".so") else LIB
    subs = [a for a in sys.argv[1:] if not a.endswith(".so")] or ["sweep_kernel"]
    for name, meta in sorted(kernels(lib).items()):
        if any(s in name for s in subs):
            regs, scratch, vsp, ssp = budget(meta)
            print(f"{name}: vgpr+agpr {regs} scratch {scratch} B vgpr_spill {vsp} sgpr_spill {ssp} "
                  f"lds {meta['.group_segment_fixed_size']} B")


if __name__ == "__main__":
    main()
