"""Per-kernel register / scratch / occupancy report of the gfx950 code objects
embedded in libheat2d.so (no GPU needed).

The shared library carries one clang offload bundle per HIP translation unit
in its .hip_fatbin section; each holds an amdgcn ELF whose AMDGPU metadata note
lists every kernel's VGPR / AGPR / SGPR counts and private (scratch) segment
size. `llvm-readelf --notes` prints that note; this module extracts the code
objects and parses it.

    python tools/isa_report.py [path/to/libheat2d.so] [--filter tb_kernel]
"""
import os
import re
import struct
import subprocess
import sys
import tempfile

READELF = "/opt/rocm/lib/llvm/bin/llvm-readelf"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def code_objects(so_path):
    """Yield (triple, bytes) of every amdgcn code object in the library."""
    data = open(so_path, "rb").read()
    pos = data.find(MAGIC)
    while pos >= 0:
        n = struct.unpack_from("<Q", data, pos + 24)[0]
        p = pos + 32
        for _ in range(n):
            off, size, tlen = struct.unpack_from("<QQQ", data, p)
            triple = data[p + 24:p + 24 + tlen].decode()
            p += 24 + tlen
            if "amdgcn" in triple and size > 0:
                yield triple, data[pos + off:pos + off + size]
        pos = data.find(MAGIC, pos + 32)


def kernels(so_path):
    """List of dicts: name, vgpr, agpr, sgpr, scratch, waves_per_simd (VGPR-limited)."""
    out = []
    with tempfile.TemporaryDirectory() as td:
        for i, (triple, blob) in enumerate(code_objects(so_path)):
            f = os.path.join(td, f"co{i}.o")
            open(f, "wb").write(blob)
            txt = subprocess.run([READELF, "--notes", f], capture_output=True, text=True, check=True).stdout
            # one metadata map per kernel, keys in alphabetical order:
            # .agpr_count ... .name ... .private_segment_fixed_size ... .vgpr_count
            for m in re.finditer(r"\.name:\s+(\S+)", txt):
                name = m.group(1)
                if name.endswith(".kd") or not name.startswith("_Z"):
                    continue
                end = txt.find(".vgpr_count", m.end())
                end = txt.find("\n", end) if end >= 0 else len(txt)
                start = txt.rfind(".agpr_count", 0, m.start())
                block = txt[start if start >= 0 else m.start():end]

                def field(key, default=0, block=block):
                    f = re.search(r"\." + key + r":\s+(\d+)", block)
                    return int(f.group(1)) if f else default
                vg, ag = field("vgpr_count"), field("agpr_count")
                # unified register file: 512 per SIMD lane, 8-register granule;
                # on gfx90a+ .vgpr_count is the TOTAL (arch VGPRs aligned to 4,
                # then the AGPRs: fp64 K = 20 general kernel 374 = 256 + 118)
                regs = ((vg + 7) // 8) * 8
                out.append({"name": name, "triple": triple, "vgpr": vg, "agpr": ag,
                            "sgpr": field("sgpr_count"), "scratch": field("private_segment_fixed_size"),
                            "waves_per_simd": min(8, 512 // max(regs, 1))})
    return out


_TB = re.compile(r"tb_kernelI([df])Li(\d+)ELi(\d+)ELi(\d+)ELb([01])ELi(\d+)E(?:Li(\d)E)?")


def tb_params(mangled):
    """(dtype, NV, K, RING, MAIN, AR) of a tb_kernel instance, or None."""
    m = _TB.search(mangled)
    if not m:
        return None
    p = ("fp64" if m.group(1) == "d" else "fp32", int(m.group(2)), int(m.group(3)), int(m.group(4)),
         m.group(5) == "1", int(m.group(6)))
    var = m.group(7) or "0"  # kernel variant (tb_impl.hpp): 1 fused statistics
    return p + ({"1": "stats"}.get(var, "var" + var),) if var != "0" else p


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    filt = "tb_kernel"
    if "--filter" in sys.argv:
        filt = sys.argv[sys.argv.index("--filter") + 1]
        args = [a for a in args if a != filt]
    so = args[0] if args else os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                           "cuda-hip-mpi-heat-equation-test_amd", "_native", "libheat2d.so")
    for k in kernels(so):
        if filt not in k["name"]:
            continue
        p = tb_params(k["name"])
        tag = (f"tb_kernel<{p[0]}, NV={p[1]}, K={p[2]:2d}, RING={p[3]}, {'main' if p[4] else 'gen '}, "
               f"{('exact', 'fma', 'jacobi', 'fast')[p[5]]}{', ' + p[6] if len(p) > 6 else ''}>") if p else k["name"][:60]
        print(f"{tag:55s} vgpr {k['vgpr']:3d} agpr {k['agpr']:3d} scratch {k['scratch']:4d} "
              f"waves/SIMD {k['waves_per_simd']}")


if __name__ == "__main__":
    main()
