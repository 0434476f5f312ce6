"""Achievable VALU issue rate of a scoring kernel from its instruction mix.

The VALU "peak" bench.py quotes by default assumes every wave64 VALU instruction issues in 2
cycles per SIMD.  The microbenchmark profiles/r01/valu_rate_gfx950.txt shows that holds only
for plain VOP1/VOP2 operations (add, and, shifts, f32 add: 2.1-2.5 cycles); VOP3-only
operations (min3, bfe, add3, lshl_add, perm, packed 16-bit ops, v_pk_minimum3_f16, compares,
SDWA / DPP forms) take 4.1-4.5 cycles, f64 operations 4.  This script disassembles the
gfx950 code object of libdukehip.so, takes the kernel's innermost loop bodies (backward
branches), prices each VALU instruction by that table and reports the mix-weighted cycles per
instruction -- a static estimate: the hot loops dominate the dynamic count, but trip counts are
not weighted.

usage: python scripts/valu_mix.py [libdukehip.so] > profiles/valu_mix.json
"""
import json
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LLVM = "/opt/rocm/lib/llvm/bin"
KERNELS = {  # bench.py roofline pmc_key -> (the kernel its launches use, loop region priced)
    # "inner": the innermost loop bodies (the DP kernels' cell loops); "outer": the largest
    # loop body (k_score_gq's per-group loop, whose inner loops are rare tails)
    "dedup": ("_ZN2dk12k_score_sym2ILi40E", "inner"),  # two queries per wave (k_score_sym2)
    "dedup_utf16": ("_ZN2dk7k_scoreILi40ELb1ELb0E", "inner"),
    "linkage": ("_ZN2dk10k_score_gqILi2ELi2ELi0E", "outer"),   # role 0 deferred (the build's default)
    "allpairs_lev": ("_ZN2dk7k_scoreILi16ELb0ELb0E", "inner"),
    "allpairs_jw": ("_ZN2dk7k_scoreILi16ELb0ELb0E", "inner"),
    "longtext": ("_ZN2dk12k_score_longILi16ELi16E", "inner"),
    "reference": ("_ZN2dk7k_scoreILi16ELb0ELb0E", "inner"),
}
# cycles per wave64 instruction per SIMD (profiles/r01/valu_rate_gfx950.txt), by class
TWO = ("v_add_u32_e32", "v_sub_u32_e32", "v_subrev_u32_e32", "v_and_b32_e32", "v_or_b32_e32",
       "v_xor_b32_e32", "v_lshrrev_b32_e32", "v_lshlrev_b32_e32", "v_ashrrev_i32_e32",
       "v_add_f32_e32", "v_min_u16_e32", "v_add_u16_e32", "v_mov_b32_e32", "v_not_b32_e32",
       "v_bitop3_b32", "v_mul_f32_e32", "v_min_i32_e32", "v_max_i32_e32")


def cycles(op):
    if op in TWO:
        return 2.3
    if "_f64" in op:
        return 4.0
    if op.startswith("v_cndmask"):
        return 4.0   # the microbenchmark's 22.8 is a VCC-dependency artefact of its loop
    return 4.2       # VOP3-only / e64 / SDWA / DPP / packed / compares


def function_body(dis, sym):
    lines = dis.splitlines()
    start = next(i for i, l in enumerate(lines) if re.match(rf"^[0-9a-f]+ <{re.escape(sym)}", l))
    body = []
    for l in lines[start + 1:]:
        if re.match(r"^[0-9a-f]+ <", l):
            break
        body.append(l)
    return body


def innermost_loops(body):
    ins = []
    for l in body:
        m = re.match(r"^\s+(\S+)\s*(.*?)\s*//\s*([0-9A-Fa-f]+):", l)
        if m:
            ins.append((int(m.group(3), 16), m.group(1), l))
    loops = []
    base = ins[0][0]  # branch targets are printed relative to the function symbol
    for addr, op, l in ins:
        if op.startswith("s_cbranch") or op == "s_branch":
            t = re.search(r"<[^>]*\+0x([0-9a-f]+)>", l)
            if t:
                tgt = base + int(t.group(1), 16)
                if tgt <= addr:
                    loops.append((tgt, addr))
    inner = [a for a in loops if not any(b != a and a[0] <= b[0] and b[1] <= a[1] for b in loops)]
    return ins, inner


def all_loops(ins):
    base = ins[0][0]
    loops = []
    for addr, op, l in ins:
        if op.startswith("s_cbranch") or op == "s_branch":
            t = re.search(r"<[^>]*\+0x([0-9a-f]+)>", l)
            if t and base + int(t.group(1), 16) <= addr:
                loops.append((base + int(t.group(1), 16), addr))
    return loops


def mix(dis, sym, region="inner"):
    ins, inner = innermost_loops(function_body(dis, sym))
    if region == "outer":  # the single largest loop (backward branch spanning the most code)
        spans = all_loops(ins)
        inner = [max(spans, key=lambda a: a[1] - a[0])] if spans else []
    counts = {}
    for lo, hi in inner:
        for addr, op, _ in ins:
            if lo <= addr <= hi and op.startswith("v_") and not op.startswith(("v_readfirstlane", "v_readlane", "v_writelane")):
                counts[op] = counts.get(op, 0) + 1
    n = sum(counts.values())
    cyc = sum(cycles(op) * c for op, c in counts.items())
    return {"kernel": sym, "region": region, "loops": len(inner), "valu_static": n,
            "avg_cycles_per_valu": cyc / n if n else None,
            "two_cycle_frac": sum(c for op, c in counts.items() if cycles(op) < 3) / n if n else None,
            "top": sorted(counts.items(), key=lambda kv: -kv[1])[:12]}


def main():
    lib = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "sesam-duke-microservice_amd", "build",
                                                           "libdukehip.so")
    with tempfile.TemporaryDirectory() as d:
        local = os.path.join(d, "lib.so")   # the bundles are written next to the input
        with open(lib, "rb") as a, open(local, "wb") as b:
            b.write(a.read())
        subprocess.run([f"{LLVM}/llvm-objdump", "--offloading", local], cwd=d, check=True,
                       capture_output=True)
        # one code object per translation unit (dk_kernels, dk_score_grouped, dk_grams)
        dis = "".join(subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn", os.path.join(d, co)],
                                     check=True, capture_output=True, text=True).stdout
                      for co in sorted(os.listdir(d)) if "gfx950" in co)
    out = {"source": "static mix of each kernel's priced loop region; cycle table "
                     "profiles/r01/valu_rate_gfx950.txt"}
    commit = os.environ.get("DK_COMMIT") or subprocess.run(
        ["git", "rev-parse", "--short", "HEAD"], cwd=ROOT, capture_output=True, text=True).stdout.strip()
    for w, (k, region) in KERNELS.items():
        sym = re.search(rf"<({re.escape(k)}[^>]*)>:", dis)
        if sym:
            out[w] = dict(mix(dis, sym.group(1), region), commit=commit)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
