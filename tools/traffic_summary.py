"""Per-launch HBM traffic of the roofline kernels from tools/pmc_traffic.sh output (JSON on stdout).

Counters are summed per dispatch over the kernel's instances (FETCH_SIZE / WRITE_SIZE, KB) and
averaged over the dispatches of the phase's timed kernel; PyTorch's own kernels (input generation)
are excluded.  Correction (MI355X_MICROARCH.md, HBM): FETCH_SIZE reports half the bytes of 16-B/lane
streaming reads; other widths are uncalibrated, so the dword-access correction is calibrated here on
the causal conv forward, whose bytes are known exactly (reads x once, writes out once: 4 B each per
element), and applied to the dword-access kernels (scan, dwconv, cconv).  MIOpen's conv kernels and the dilated-conv
weight gradient (float4 buffer loads) use wide loads: the documented x2 applies.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

root = sys.argv[1]
SHAPES = {"scan": (64, 1024, 3999), "scan_bwd": (64, 1024, 3999), "dwconv": (16, 512, 3999), "cconv": (64, 1024, 3999),
          "conv3": (32, 64, 376, 257), "dconv_wgrad": (32, 64, 376, 257),
          "scan_c5": (32, 1024, 5999), "scan_bwd_c5": (32, 1024, 5999),
          "dwconv_gln": (16, 512, 3999), "dwconv_gln_bwd": (16, 512, 3999),
          "prelu_gln": (16, 512, 3999), "prelu_gln_bwd": (16, 512, 3999)}


# the kernels one call of a multi-launch op consists of (name substrings); other phases: the dominant kernel.  A bwd
# phase's setup call of the forward runs the forward's kernels once — they are not in these sets
OPS = {"scan_bwd": ("scan::bwd_kernel", "scan::reduce_bc_kernel", "scan::reduce_d_kernel"),
       "scan_bwd_c5": ("scan::bwd_kernel", "scan::reduce_bc_kernel", "scan::reduce_d_kernel"),
       "dwconv_gln": ("gln::dwconv_stats_kernel", "gln::apply_fused_kernel"),
       "dwconv_gln_bwd": ("gln::bwd_reduce_kernel", "gln::dwconv_gln_bwd", "gln::dw_tail_kernel"),
       "prelu_gln": ("gln::stats_kernel", "gln::apply_fused_kernel"),
       "prelu_gln_bwd": ("gln::bwd_reduce_kernel", "gln::bwd_apply_kernel", "gln::bwd_finalize",
                         "gln::alpha_finalize")}


def per_launch(phase, counter):
    """(bytes per call of the phase's op, kernel label): the per-dispatch average of each of the op's kernels,
    summed over them (OPS), or of the dominant kernel alone."""
    f = glob.glob(os.path.join(root, phase, counter, "**", "*counter_collection.csv"), recursive=True)
    if not f:
        return None, None
    per = defaultdict(float)
    names = {}
    for r in csv.DictReader(open(f[0])):
        name = r["Kernel_Name"]
        if "at::native" in name or "at::" in name[:12]:
            continue
        per[r["Dispatch_Id"]] += float(r["Counter_Value"])
        names[r["Dispatch_Id"]] = name
    if not per:
        return None, None

    def avg(n):
        vals = [per[d] for d in per if names[d] == n]
        return sum(vals) / len(vals)
    if phase in OPS:
        ks = sorted({n for n in names.values() if any(p in n for p in OPS[phase])})
        return sum(avg(n) for n in ks) * 1024.0, " + ".join(k.split("(")[0].replace("void ", "") for k in ks)
    kern = max(set(names.values()), key=lambda n: sum(per[d] for d in per if names[d] == n))
    return avg(kern) * 1024.0, kern.split("(")[0]     # KB -> bytes


res = {}
raw = {ph: {c: per_launch(ph, c) for c in ("FETCH_SIZE", "WRITE_SIZE")} for ph in SHAPES
       if os.path.isdir(os.path.join(root, ph))}
b, d, l = SHAPES["cconv"]
known = 4.0 * b * d * l
cal_src = "this run's cconv phase"
if "cconv" in raw:
    cal_r = known / raw["cconv"]["FETCH_SIZE"][0] if raw["cconv"]["FETCH_SIZE"][0] else None
    cal_w = known / raw["cconv"]["WRITE_SIZE"][0] if raw["cconv"]["WRITE_SIZE"][0] else None
else:       # a run of some phases only: the dword corrections of an earlier run's calibration (CAL_FROM=traffic.json)
    cal_src = os.environ["CAL_FROM"]
    prev = json.load(open(cal_src))["calibration"]
    cal_r, cal_w = prev["dword_read_correction"], prev["dword_write_correction"]
for ph in raw:
    fr, kern = raw[ph]["FETCH_SIZE"]
    wr, _ = raw[ph]["WRITE_SIZE"]
    if fr is None or wr is None:
        continue
    rf, wf = (2.0, 1.0) if ph in ("conv3", "dconv_wgrad") else (cal_r, cal_w)     # 16-B/lane loads: the documented x2
    res[ph] = {"kernel": kern, "fetch_bytes": round(fr * rf), "write_bytes": round(wr * wf),
               "traffic_bytes": round(fr * rf + wr * wf), "raw_fetch_size_bytes": round(fr), "raw_write_size_bytes": round(wr),
               "read_correction": round(rf, 4), "write_correction": round(wf, 4)}
res["calibration"] = {"kernel": "avse_cconv_fwd (B=64, D=1024, L=3999): reads x once, writes out once",
                      "known_read_bytes": known, "known_write_bytes": known,
                      "dword_read_correction": cal_r, "dword_write_correction": cal_w, "source": cal_src}
print(json.dumps(res, indent=1))
