#!/usr/bin/env python3
"""Per-launch HBM traffic of one kernel from rocprofv3 --pmc CSVs (FETCH_SIZE and
WRITE_SIZE collected in separate passes), corrected as MI355X_MICROARCH.md §HBM
prescribes: counters are in KiB; on gfx950 FETCH_SIZE reads exactly half the bytes
of a wide (16 B/lane) coalesced streaming read, so it is doubled; WRITE_SIZE is
exact for 16-B-per-lane streaming stores (our 2-4 B/lane column stores are
uncalibrated: reported as-is).

  python tools/pmc_summary.py <fetch_dir> <write_dir> <kernel-substring> <out.json> [alg_bytes]
"""
import csv
import glob
import json
import statistics
import sys


def values(d, counter, kname):
    out = []
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter and kname in r["Kernel_Name"]:
                out.append(float(r["Counter_Value"]))
    return out


def main():
    fdir, wdir, kname, out = sys.argv[1:5]
    alg = float(sys.argv[5]) if len(sys.argv) > 5 else None
    fetch = values(fdir, "FETCH_SIZE", kname)
    write = values(wdir, "WRITE_SIZE", kname)
    if not fetch or not write:
        raise SystemExit(f"no samples for {kname}: fetch={len(fetch)} write={len(write)}")
    f_kib, w_kib = statistics.median(fetch), statistics.median(write)
    read_b = 2.0 * f_kib * 1024
    write_b = w_kib * 1024
    d = {"kernel": kname, "launches": [len(fetch), len(write)],
         "FETCH_SIZE_kib_median": f_kib, "WRITE_SIZE_kib_median": w_kib,
         "read_bytes_per_launch": read_b, "write_bytes_per_launch": write_b,
         "hbm_bytes_per_launch": read_b + write_b,
         "correction": "FETCH_SIZE x2 (gfx950 wide-streaming-read undercount), KiB->bytes x1024",
         "alg_bytes_per_launch": alg,
         "traffic_over_alg": (read_b + write_b) / alg if alg else None}
    json.dump(d, open(out, "w"), indent=1)
    print(json.dumps(d))


if __name__ == "__main__":
    main()
