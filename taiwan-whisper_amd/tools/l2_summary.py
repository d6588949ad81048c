"""Summary of tools/gpu_r4b.sh: per shape and tile order, FETCH_SIZE bytes per launch (x 1024 x 2: the counter is
in KiB and reads half the bytes of 16-B streaming loads on gfx950, MI355X_MICROARCH.md §HBM; Infinity-Cache hits
included) against the algorithmic bytes (A + B read once, C written once), and the L2 hit rate."""
import csv
import glob
import os
import sys


def per_launch(d, counter):
    vals = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter and "gemm" in r["Kernel_Name"]:
                vals.append(float(r["Counter_Value"]))
    vals = vals[1:] if len(vals) > 1 else vals          # the first launch also warms the caches
    return sum(vals) / len(vals) if vals else float("nan")


def main():
    out = sys.argv[1]
    for f in sorted(glob.glob(os.path.join(out, "f_*_g*"))):
        tag = os.path.basename(f)[2:]
        shape, g = tag.rsplit("_g", 1)
        M, N, K = map(int, shape.split("_"))
        fetch = per_launch(f, "FETCH_SIZE") * 1024 * 2
        hit = per_launch(os.path.join(out, "h_" + tag), "TCC_HIT_sum")
        miss = per_launch(os.path.join(out, "h_" + tag), "TCC_MISS_sum")
        algo_rd = 2.0 * (M * K + N * K)
        print(f"M={M:6d} N={N:6d} K={K:5d} group {g}: fetch {fetch/1e9:7.3f} GB = {fetch/algo_rd:5.2f}x algorithmic "
              f"reads ({algo_rd/1e9:.3f} GB)  L2 hit {hit/(hit+miss):.3f}")


if __name__ == "__main__":
    main()
