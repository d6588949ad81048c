"""Per-kernel summary of a rocprofv3 kernel-trace database (rocpd SQLite, ROCm 7 default output).

    python tools/rocpd_stats.py gpurun_out/prof/run_results.db [--steps 3] [--csv out.csv]

Prints name, calls, total ms, avg us, share of GPU time, and ms per step (total / --steps), i.e.
the same columns as `rocprofv3 --stats` kernel_stats.csv plus the per-step view used in DESIGN.md.
Grid/workgroup sizes are kept so that tile variants of one template are told apart.
"""
import argparse
import collections
import glob
import os
import sqlite3


def load(db):
    c = sqlite3.connect(db)
    tabs = [r[0] for r in c.execute("select name from sqlite_master where type='table'")]
    ks = next(t for t in tabs if t.startswith("rocpd_info_kernel_symbol"))
    kd = next(t for t in tabs if t.startswith("rocpd_kernel_dispatch"))
    q = (f"select s.display_name, d.start, d.end, d.workgroup_size_x, s.group_segment_size, "
         f"s.arch_vgpr_count from {kd} d join {ks} s on d.kernel_id = s.id")
    return list(c.execute(q))


def summarize(rows, short=True):
    agg = collections.defaultdict(lambda: [0, 0])
    for name, t0, t1, wg, lds, vgpr in rows:
        n = name.replace("(anonymous namespace)::", "").replace("void ", "", 1)
        if short:
            depth, cut = 0, len(n)
            for i, ch in enumerate(n):      # first '(' outside template brackets = the parameter list
                depth += (ch == "<") - (ch == ">")
                if ch == "(" and depth == 0:
                    cut = i
                    break
            n = n[:cut]
        key = f"{n} [wg{wg} lds{lds // 1024}K v{vgpr}]"
        agg[key][0] += 1
        agg[key][1] += t1 - t0
    return agg


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--steps", type=float, default=1.0)
    ap.add_argument("--csv", default=None)
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    db = a.db if a.db.endswith(".db") else glob.glob(os.path.join(a.db, "**", "*.db"), recursive=True)[0]
    agg = summarize(load(db))
    tot = sum(v[1] for v in agg.values())
    items = sorted(agg.items(), key=lambda kv: -kv[1][1])
    lines = ["Name,Calls,TotalMs,AverageUs,Percentage,MsPerStep"]
    for k, (n, ns) in items:
        lines.append(f"\"{k}\",{n},{ns / 1e6:.3f},{ns / n / 1e3:.2f},{100 * ns / tot:.2f},{ns / 1e6 / a.steps:.3f}")
    if a.csv:
        with open(a.csv, "w") as f:
            f.write("\n".join(lines) + "\n")
    print(f"total GPU kernel time {tot / 1e6:.1f} ms ({tot / 1e6 / a.steps:.1f} ms/step over {a.steps:g} steps)")
    for ln in lines[: a.top + 1]:
        print(ln)


if __name__ == "__main__":
    main()
