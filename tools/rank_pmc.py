"""Fabric traffic of a frame split into rank lists against the whole frame (tooling).

Reads the counter_collection.csv of a `rocprofv3 --pmc FETCH_SIZE` (and one of
WRITE_SIZE) run of tools/rank_sim.py and prints, per (march kernel, grid size),
the mean traffic per dispatch -- 2 x FETCH_SIZE + WRITE_SIZE KiB, the gfx950
correction of MI355X_MICROARCH.md used by tools/pmc_traffic.py -- so the sum
over a split's ranks can be set against the full frame's.

  python tools/rank_pmc.py FETCH.csv WRITE.csv
"""
import collections
import csv
import sys


def per_dispatch(path, counter):
    acc = collections.defaultdict(list)
    for row in csv.DictReader(open(path)):
        if row["Counter_Name"] != counter or "vr::k_march" not in row["Kernel_Name"]:
            continue
        name = row["Kernel_Name"].split("(")[0].replace("void ", "")
        acc[(name, int(row["Grid_Size"]))].append(float(row["Counter_Value"]))
    return {k: (sum(v) / len(v), len(v)) for k, v in acc.items()}


def main():
    fetch = per_dispatch(sys.argv[1], "FETCH_SIZE")
    write = per_dispatch(sys.argv[2], "WRITE_SIZE") if len(sys.argv) > 2 else {}
    for key in sorted(fetch, key=lambda k: -k[1]):
        f, n = fetch[key]
        w = write.get(key, (0.0, 0))[0]
        gb = (2.0 * f + w) * 1024.0 / 1e9
        print(f"{key[0]:45s} grid {key[1]:9d}  dispatches {n:4d}  traffic {gb:7.3f} GB/dispatch")


if __name__ == "__main__":
    main()
