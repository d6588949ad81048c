"""Per-(kernel, grid) summary of a rocprofv3 --kernel-trace --output-format csv run, so that the
shapes of one kernel template are told apart.  usage: trace_by_grid.py <dir> [--reps N] [--skip-first K]"""
import argparse
import collections
import csv
import glob
import os


def short(n):
    n = n.replace("(anonymous namespace)::", "").replace("void ", "", 1)
    depth = 0
    for i, ch in enumerate(n):
        depth += (ch == "<") - (ch == ">")
        if ch == "(" and depth == 0:
            return n[:i]
    return n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--reps", type=float, default=1.0)
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    f = glob.glob(os.path.join(a.dir, "**", "*kernel_trace.csv"), recursive=True)[0]
    agg = collections.defaultdict(lambda: [0, 0])
    for r in csv.DictReader(open(f)):
        key = (short(r["Kernel_Name"]), f'{r["Grid_Size_X"]}x{r["Grid_Size_Y"]}x{r["Grid_Size_Z"]}/{r["Workgroup_Size_X"]}')
        agg[key][0] += 1
        agg[key][1] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    tot = sum(v[1] for v in agg.values())
    print(f"total {tot / 1e6:.1f} ms, {tot / 1e6 / a.reps:.2f} ms per rep")
    for (n, g), (c, ns) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:a.top]:
        print(f"{ns / 1e6 / a.reps:9.3f} ms/rep {100 * ns / tot:5.1f}%  {c:5d}x {ns / c / 1e3:9.1f}us  {n[:70]}  {g}")


if __name__ == "__main__":
    main()
