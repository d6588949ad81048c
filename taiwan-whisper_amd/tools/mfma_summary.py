"""MFMA-busy summary per kernel family from a rocprofv3 --pmc pass with SQ_VALU_MFMA_BUSY_CYCLES,
GRBM_GUI_ACTIVE and SQ_BUSY_CYCLES (one pass: 2 SQ + 1 GRBM counters).

Units (MI355X_MICROARCH.md, cycle constants / DVFS): SQ_VALU_MFMA_BUSY_CYCLES adds each MFMA's
busy cycles on its SIMD (32 per v_mfma_f32_32x32x16_bf16, 16 per 16x16x32), summed over the chip;
GRBM_GUI_ACTIVE is the sum over the 8 XCDs of the cycles the GPU was busy.  So for a dispatch
    MFMA-busy fraction = MFMA_BUSY / (GRBM_GUI_ACTIVE / 8 * 1024 SIMDs)
(the share of SIMD-cycles spent issuing matrix work, at whatever clock the chip held), and
1024 * MFMA_BUSY = bf16 FLOPs the matrix cores executed (1024 FLOP per SIMD-cycle for both bf16 shapes;
padding included), a check on the algorithmic FLOPs.

"other" = kernels outside the named families (torch fills / random init of the benchmark models, embedding,
small elementwise); ALL_BUT_OTHER is the forward / step kernels proper.

usage: python mfma_summary.py <pmc_dir> [label] [--json out.json]
"""
import collections
import csv
import glob
import json
import os
import re
import sys

FAMILIES = [
    ("gemm_pp (persistent 256x256 forward GEMM)", r"gemm_pp_kernel"),
    ("gemm 128x128 / 256 tiles (small-grid fwd, dX, dW)", r"gemm_kernel<"),
    ("gemm skinny (decode)", r"gemm_skinny"),
    ("hipBLASLt (plain projections)", r"Cijk_"),
    ("attention fwd", r"attn_fwd"),
    ("attention bwd", r"attn_bwd"),
    ("fp32 gemm", r"gemm_f32|f32_gemm"),
    ("layernorm", r"ln_fwd|ln_bwd"),
    ("klce", r"klce"),
    ("logmel", r"logmel"),
]


def load(d):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]
    per = collections.defaultdict(dict)
    names = {}
    for r in csv.DictReader(open(f)):
        did = r.get("Dispatch_Id") or r.get("Correlation_Id")
        per[did][r["Counter_Name"]] = per[did].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        per[did]["ns"] = float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
        names[did] = r["Kernel_Name"]
    return per, names


def summarize(d):
    per, names = load(d)
    fam = collections.defaultdict(lambda: [0, 0.0, 0.0, 0.0, 0.0])
    for did, c in per.items():
        n = names[did]
        key = next((k for k, pat in FAMILIES if re.search(pat, n)), "other")
        f = fam[key]
        f[0] += 1
        f[1] += c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0)
        f[2] += c.get("GRBM_GUI_ACTIVE", 0.0)
        f[3] += c.get("SQ_BUSY_CYCLES", 0.0)
        f[4] += c.get("ns", 0.0)
    out = {}
    tot = collections.defaultdict(lambda: [0, 0.0, 0.0, 0.0])
    for k, (n, mb, grbm, sqb, ns) in sorted(fam.items(), key=lambda kv: -kv[1][2]):
        frac = mb / (grbm / 8 * 1024) if grbm else 0.0
        out[k] = dict(dispatches=n, mfma_busy_cycles=mb, grbm_gui_active=grbm, sq_busy_cycles=sqb, kernel_ms=ns / 1e6,
                      mfma_busy_frac=round(frac, 4), mfma_tflop_executed=round(mb * 1024 / 1e12, 3),
                      effective_clock_ghz=round(grbm / 8 / ns, 3) if ns else None, share_of_gpu_cycles=None)
        for t in (("ALL",) if k == "other" else ("ALL", "ALL_BUT_OTHER")):
            tot[t][0] += n
            tot[t][1] += mb
            tot[t][2] += grbm
            tot[t][3] += ns
    for k in out:
        out[k]["share_of_gpu_cycles"] = round(out[k]["grbm_gui_active"] / tot["ALL"][2], 4) if tot["ALL"][2] else None
    for t, (n, mb, grbm, ns) in tot.items():
        out[t] = dict(dispatches=n, mfma_busy_frac=round(mb / (grbm / 8 * 1024), 4) if grbm else 0.0,
                      mfma_tflop_executed=round(mb * 1024 / 1e12, 3), kernel_ms=ns / 1e6,
                      effective_clock_ghz=round(grbm / 8 / ns, 3) if ns else None)
    return out


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    js = sys.argv[sys.argv.index("--json") + 1] if "--json" in sys.argv else None
    d = args[0]
    label = args[1] if len(args) > 1 else d
    out = summarize(d)
    print(f"== {label}: MFMA-busy fraction = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE/8 x 1024 SIMDs)")
    for k, v in out.items():
        print(f"  {k:52s} {v['dispatches']:6d} disp  mfma_busy {v['mfma_busy_frac']:.3f}  "
              f"executed {v['mfma_tflop_executed']:9.2f} TFLOP  clock {v['effective_clock_ghz']} GHz" + (
                  f"  share of GPU cycles {v['share_of_gpu_cycles']:.3f}" if v.get("share_of_gpu_cycles") else ""))
    if js:
        with open(js, "w") as f:
            json.dump({label: out}, f, indent=1)


if __name__ == "__main__":
    main()
