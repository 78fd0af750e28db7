"""HBM bytes per launch of the march kernel from rocprofv3 PMC passes (tooling).

Counters are collected in separate passes (FETCH_SIZE costs 3 of the 4 TCC slots,
WRITE_SIZE 2; MI355X_MICROARCH.md "rocprofv3 PMC slots"), each pass a full
`bench.py` run under `rocprofv3 --pmc ... --output-format csv`.  Corrections per
the guide's HBM section:
  * FETCH_SIZE is tallied as TCC_EA0_RDREQ x 64 B although gfx950 issues 128-B
    memory-side reads for wide streaming loads -> the read bytes are
    2 x FETCH_SIZE.  The raw EA request counts are recorded beside it so the
    factor can be checked against TCC_EA0_RDREQ (pass 3).
  * WRITE_SIZE is taken as is.
  * Infinity-Cache (MALL) hits are counted by these fabric-side counters, so
    the figure is an upper bound on DRAM bytes.
FETCH_SIZE / WRITE_SIZE are reported by rocprofv3 in KiB.

usage: python tools/pmc_traffic.py OUT.json KEY BENCH_LOG PASS_DIR [PASS_DIR ...]
  (an issue pass with SQ_INSTS_VALU / SQ_WAVES / GRBM_GUI_ACTIVE adds the VALU count)
  KEY       entry name, e.g. "1024x8|C0|m1"
  BENCH_LOG stdout of the profiled bench.py (its JSON line names the kernel)
"""
import collections
import csv
import glob
import json
import os
import sys


def per_dispatch(dirs):
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    names = {}
    grids = {}
    for d in dirs:
        for f in sorted(glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)):
            rows = collections.defaultdict(dict)
            for r in csv.DictReader(open(f)):
                k = r["Kernel_Name"]
                if "vr::k_march" not in k or ", true>" in k and ("vr::k_march<" in k or
                                                                  "vr::k_march_gmm<" in k):
                    continue  # the march only (not the footprint-counting variants)
                # a kernel is keyed with its grid: bench.py's one-tile latency probe (roofline.compute)
                # may launch the frame's own kernel on a 256-thread grid
                k = (k, int(r["Grid_Size"]))
                rows[(k, r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
                grids[k] = k[1]
            for (k, _), cs in rows.items():
                names[k] = names.get(k, 0) + 1
                for c, v in cs.items():
                    vals[k][c].append(v)
    if not names:
        raise SystemExit("no march dispatches in the PMC output")
    # the frame's launch: the largest grid (bench.py also launches a one-tile
    # latency probe, roofline.compute, several times), then the most dispatches
    kernel = max(names, key=lambda k: (grids[k], names[k]))
    return kernel[0], {c: sum(v) / len(v) for c, v in vals[kernel].items()}


def main():
    out_path, key, bench_log = sys.argv[1:4]
    kernel_full, avg = per_dispatch(sys.argv[4:])
    bench = None
    for line in open(bench_log):
        line = line.strip()
        if line.startswith("{") and '"metric"' in line:
            bench = json.loads(line)
    fetch_kib = avg.get("FETCH_SIZE")
    write_kib = avg.get("WRITE_SIZE")
    rd = avg.get("TCC_EA0_RDREQ_sum")
    entry = {
        "kernel": bench["roofline"]["kernel"] if bench else None,
        "kernel_symbol": kernel_full,
        "config": bench["config"] if bench else None,
        "fetch_size_kib": fetch_kib,
        "write_size_kib": write_kib,
        "tcc_ea0_rdreq": rd,
        "read_bytes": 2.0 * fetch_kib * 1024 if fetch_kib is not None else None,
        "write_bytes": write_kib * 1024 if write_kib is not None else None,
        "alg_bytes_per_launch": bench["roofline"]["alg_bytes_per_launch"] if bench else None,
    }
    # issue pass (optional): VALU wave-instructions per launch (SQ_INSTS_VALU counts
    # instructions on gfx950, as SQ_ACTIVE_INST_VALU does: tools/valu_calib.hip) and
    # the clock cycles of the launch (GRBM_GUI_ACTIVE summed over the 8 XCDs)
    for c, k in (("SQ_INSTS_VALU", "valu_insts"), ("SQ_INSTS_VMEM_RD", "vmem_rd_insts"),
                 ("SQ_INSTS_LDS", "lds_insts"), ("SQ_WAVES", "waves"),
                 ("GRBM_GUI_ACTIVE", "grbm_gui_active")):
        if c in avg:
            entry[k] = avg[c]
    if entry["read_bytes"] is not None and entry["write_bytes"] is not None:
        entry["hbm_bytes_per_launch"] = int(entry["read_bytes"] + entry["write_bytes"])
    # the build the passes ran on: bench.py reports this traffic only for it
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import bench as _bench
    lib = os.environ.get("VRDD_LIB") or os.path.join(
        root, "volume-rendering-based-on-distribution-data_amd", "csrc", "build", "libvr.so")
    entry["lib_sha16"] = _bench.lib_sha16(lib)
    entry["measured"] = os.environ.get("PMC_TAG", "")
    db = {}
    if os.path.exists(out_path):
        db = json.load(open(out_path))
    db[key] = entry
    with open(out_path, "w") as f:
        json.dump(db, f, indent=1, sort_keys=True)
    print(json.dumps({key: entry}))


if __name__ == "__main__":
    main()
