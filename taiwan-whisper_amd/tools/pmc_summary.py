"""Per-kernel-family HBM traffic from two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE).

gfx950 corrections (MI355X_MICROARCH.md §HBM): FETCH_SIZE/WRITE_SIZE are in KiB; FETCH_SIZE reads
exactly 1/2 of the bytes of a wide (16 B/lane) coalesced streaming read -> doubled here (every tw
kernel stages operands with 16-B buffer_load ... lds); WRITE_SIZE is exact for 16-B stores (bf16x4
8-B stores are uncalibrated).  Infinity-Cache hits appear to be counted, so this is an upper bound
of DRAM bytes.

No counter on gfx950 splits Infinity-Cache (MALL) hits from HBM reads: TCC_EA0_RDREQ_DRAM_sum equals
TCC_EA0_RDREQ_sum for every kernel family (measured r02, share 1.000 - the request is counted before the
MALL), so the former dram_* fields were copies of the fetch and are no longer reported.  The figures are
L2-miss traffic (the L2 <-> fabric bytes), an upper bound of DRAM bytes.

usage: python pmc_summary.py <fetch_dir> <write_dir> <out.json>
"""
import csv
import json
import re
import sys
from collections import defaultdict

FAMILIES = {
    "gemm_nn": r"gemm_kernel<false, false|gemm_pp_kernel",
    "gemm_nt": r"gemm_kernel<false, true",
    "gemm_tt": r"gemm_kernel<true, true",
    "attn_fwd": r"attn_fwd_kernel",
    "klce": r"klce_kernel",
    "ln_fwd": r"ln_fwd_kernel",
    "logmel": r"logmel_kernel",
}


def load(d, counter):
    per = defaultdict(list)
    for r in csv.DictReader(open(f"{d}/run_counter_collection.csv")):
        if r["Counter_Name"] != counter:
            continue
        for fam, pat in FAMILIES.items():
            if re.search(pat, r["Kernel_Name"]):
                per[fam].append(float(r["Counter_Value"]))
    return per


def main():
    fdir, wdir, out = sys.argv[1:4]
    tag = sys.argv[4] if len(sys.argv) > 4 else "latest"
    fetch, write = load(fdir, "FETCH_SIZE"), load(wdir, "WRITE_SIZE")
    res = {"source": f"bash taiwan-whisper_amd/tools/profile_round.sh {tag} (profiles/{tag}_pmc.json)"}
    for fam in FAMILIES:
        if not fetch.get(fam) or not write.get(fam):
            continue
        f = sum(fetch[fam]) / len(fetch[fam]) * 1024 * 2
        w = sum(write[fam]) / len(write[fam]) * 1024
        res[fam] = dict(launches=len(fetch[fam]), fetch_bytes_per_launch=f, write_bytes_per_launch=w,
                        hbm_bytes_per_launch=f + w)
        print(f"{fam:9s} launches={len(fetch[fam]):5d} fetch {f/1e6:9.1f} MB  write {w/1e6:9.1f} MB per launch")
    res["_note"] = ("rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate passes over `bench.py --steps 2 --warmup 1`; "
                    "FETCH_SIZE x2 (gfx950 wide-read correction), KiB -> bytes.  L2-miss (L2 <-> fabric) bytes: "
                    "Infinity-Cache hits are counted too and no gfx950 counter separates them, so hbm_bytes_per_launch "
                    "is an upper bound of DRAM bytes")
    json.dump(res, open(out, "w"), indent=1)


if __name__ == "__main__":
    main()
