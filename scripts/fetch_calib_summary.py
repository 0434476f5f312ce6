"""FETCH_SIZE calibration summary from a raw rocprofv3 capture of scripts/micro/fetch_calib.

usage: python scripts/fetch_calib_summary.py CAPTURE_DIR OUT_JSON [source note]
  CAPTURE_DIR: rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d CAPTURE_DIR
               -o pmc -- scripts/micro/fetch_calib

Every k_read<T> launch reads exactly 2^30 bytes (one 1-GiB buffer, each byte once, far past
the Infinity Cache).  factor(W) = 2^30 / (FETCH_SIZE_KiB * 1024) for each access width W
(2, 4, 8, 16 B per lane).  A launch that reports less than 1 % of the expected bytes did not
do the work (a capture that dropped or mis-attributed it: round 4's first capture had the
u16 kernel at 9.5 KiB in 1.24 us) and is REJECTED: it is listed under "rejected" with its
figures and never enters a factor.  Exit status 1 if any width ends up without an accepted
launch, so a bad capture cannot silently produce a partial table.
"""
import collections
import csv
import glob
import json
import os
import sys

EXPECTED = 1 << 30
WIDTHS = {"unsigned short": 2, "unsigned int": 4, "unsigned long": 8, "HIP_vector_type": 16}


def width_of(kernel):
    inner = kernel[kernel.index("<") + 1:kernel.index(">")] if "<" in kernel else ""
    for k, w in WIDTHS.items():
        if inner.startswith(k):
            return w
    return None


def main():
    cap, out = sys.argv[1], sys.argv[2]
    note = sys.argv[3] if len(sys.argv) > 3 else ""
    f = glob.glob(os.path.join(cap, "**", "*counter_collection.csv"), recursive=True)
    if not f:
        sys.exit(f"no counter_collection.csv under {cap}")
    launches = collections.OrderedDict()
    for r in csv.DictReader(open(f[0])):
        if r["Counter_Name"] != "FETCH_SIZE":
            continue
        d = launches.setdefault(r["Dispatch_Id"], {"kernel": r["Kernel_Name"], "kib": 0.0})
        d["kib"] += float(r["Counter_Value"])
    # kernel durations from the trace, when present (context for a rejected launch)
    dur = {}
    for t in glob.glob(os.path.join(cap, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(t)):
            try:
                dur[r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            except (KeyError, ValueError):
                pass
    kernels, rejected = {}, []
    for disp, d in launches.items():
        w = width_of(d["kernel"])
        if w is None:
            continue
        got = d["kib"] * 1024.0
        rec = {"kernel": d["kernel"], "dispatch": int(disp), "fetch_size_kib": d["kib"],
               "duration_us": dur.get(disp)}
        if got < 0.01 * EXPECTED / 2:   # even the x2 undercount leaves >= 50 %: < 1 % is no work
            rec["reason"] = "reported < 1 % of the bytes the launch reads"
            rejected.append(rec)
            continue
        rec["factor"] = EXPECTED / got
        kernels.setdefault(f"{w}B_per_lane", rec)
    missing = [f"{w}B_per_lane" for w in (2, 4, 8, 16) if f"{w}B_per_lane" not in kernels]
    summary = {
        "source": note or f"scripts/micro/fetch_calib under rocprofv3 --kernel-trace --pmc FETCH_SIZE ({cap})",
        "bytes_read_per_kernel": EXPECTED,
        "pattern": "64 lanes read 64 consecutive elements of a row, each byte once, 1 GiB > Infinity Cache",
        "reject_rule": "a launch reporting < 1 % of its 2^30 bytes is rejected (listed, not used)",
        "kernels": {k: kernels[k] for k in sorted(kernels, key=lambda s: int(s.split("B")[0]))},
        "rejected": rejected,
        "missing_widths": missing,
    }
    with open(out, "w") as fh:
        json.dump(summary, fh, indent=1)
    print(json.dumps({k: round(v["factor"], 4) for k, v in summary["kernels"].items()}),
          "rejected", len(rejected), "missing", missing)
    if missing:
        sys.exit(1)


if __name__ == "__main__":
    main()
