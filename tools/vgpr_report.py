"""Register use of the kernels in a built libvr.so (tooling).

Splits the library's .hip_fatbin into its per-object offload bundles, unbundles
the gfx950 code objects and prints VGPR / AGPR / SGPR counts, spills and LDS
per kernel whose symbol matches the filter -- e.g. to check that a change to
the per-ray march keeps it at <= 256 VGPRs (2 waves per SIMD).

  python tools/vgpr_report.py [path/to/libvr.so] [--filter k_march_pipe]
"""
import argparse
import os
import re
import subprocess
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("lib", nargs="?", default=os.path.join(
        os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
        "volume-rendering-based-on-distribution-data_amd", "csrc", "build", "libvr.so"))
    ap.add_argument("--filter", default="k_march")
    args = ap.parse_args()
    with tempfile.TemporaryDirectory() as td:
        fat = os.path.join(td, "fat.bin")
        subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", args.lib,
                        os.path.join(td, "junk")], check=True)
        data = open(fat, "rb").read()
        offs = [m.start() for m in re.finditer(re.escape(MAGIC), data)]
        rows = []
        for k, a in enumerate(offs):
            b = offs[k + 1] if k + 1 < len(offs) else len(data)
            part, co = os.path.join(td, f"b{k}.bin"), os.path.join(td, f"b{k}.co")
            open(part, "wb").write(data[a:b])
            r = subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o",
                                "--targets=hipv4-amdgcn-amd-amdhsa--gfx950",
                                f"--input={part}", f"--output={co}"], capture_output=True)
            if r.returncode or not os.path.exists(co) or os.path.getsize(co) == 0:
                continue
            notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co],
                                   capture_output=True, text=True).stdout
            for blk in notes.split("  - .agpr_count")[1:]:
                get = lambda key: (re.search(rf"\.{key}:\s+(\S+)", blk) or [None, "?"])[1]
                name = get("name")
                if args.filter in name:
                    rows.append((name, get("vgpr_count"), "  - .agpr_count" and
                                 re.search(r"^:\s+(\d+)", blk).group(1), get("sgpr_count"),
                                 get("vgpr_spill_count"), get("sgpr_spill_count"),
                                 get("group_segment_fixed_size"),
                                 get("private_segment_fixed_size"), get("uses_dynamic_stack")))
        for name, v, a, s, vs, ss, lds, priv, dyn in sorted(set(rows)):
            print(f"{name[:90]:90s} vgpr {v:>4} agpr {a:>3} sgpr {s:>3} "
                  f"spill v{vs}/s{ss} lds {lds} private {priv}{' dynamic-stack' if dyn == 'true' else ''}")


if __name__ == "__main__":
    main()
