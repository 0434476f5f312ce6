"""Register / scratch / LDS of the gfx950 kernels in a built library (code-object metadata).

usage: python scripts/kres.py [lib.so] [kernel-name regex]
Prints per kernel: VGPRs, SGPRs, VGPR/SGPR spills, scratch bytes per lane, LDS bytes.  Reads
the AMDGPU metadata notes of every gfx950 code object (llvm-objdump --offloading +
llvm-readelf --notes): the figures `make resources` reports, without recompiling.
"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def kernels(lib):
    with tempfile.TemporaryDirectory() as d:
        local = os.path.join(d, "lib.so")
        with open(lib, "rb") as a, open(local, "wb") as b:
            b.write(a.read())
        subprocess.run([f"{LLVM}/llvm-objdump", "--offloading", local], cwd=d, check=True,
                       capture_output=True)
        notes = "".join(subprocess.run([f"{LLVM}/llvm-readelf", "--notes", os.path.join(d, co)],
                                       check=True, capture_output=True, text=True).stdout
                        for co in sorted(os.listdir(d)) if "gfx950" in co)
    out = []
    for b in notes.split("  - .agpr_count")[1:]:
        def g(k):
            m = re.search(rf"\.{k}:\s+(\S+)", b)
            return m.group(1) if m else None
        out.append({"name": g("name"), "vgpr": g("vgpr_count"), "sgpr": g("sgpr_count"),
                    "vgpr_spill": g("vgpr_spill_count"), "sgpr_spill": g("sgpr_spill_count"),
                    "scratch": g("private_segment_fixed_size"), "lds": g("group_segment_fixed_size")})
    return out


def main():
    lib = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "sesam-duke-microservice_amd", "build",
                                                           "libdukehip.so")
    rx = re.compile(sys.argv[2] if len(sys.argv) > 2 else ".")
    for k in kernels(lib):
        if k["name"] and rx.search(k["name"]):
            print(f"{k['name'][:60]:60s} vgpr {k['vgpr']:>4} sgpr {k['sgpr']:>4} vspill {k['vgpr_spill']:>3} "
                  f"sspill {k['sgpr_spill']:>3} scratch {k['scratch']:>4} lds {k['lds']}")


if __name__ == "__main__":
    main()
