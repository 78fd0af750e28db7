"""Code-object checks of the built libvr.so (CPU: reads the gfx950 kernel
metadata, runs nothing).  The LDS-box marches must use no scratch: the
round-4 k_march_duo<8,3> fault came from a register-capped
variant build whose duo spilled ~1 KB per lane to a private segment; the shipped
k_march / k_march_duo instances keep private_segment_fixed_size 0, no dynamic
stack and at most 256 VGPRs."""
import os
import re
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "volume-rendering-based-on-distribution-data_amd", "csrc", "build",
                   "libvr.so")
LLVM = "/opt/rocm/lib/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def _kernels():
    if not os.path.exists(LIB) or not os.path.exists(f"{LLVM}/llvm-readelf"):
        pytest.skip("libvr.so or the ROCm LLVM tools are absent")
    out = {}
    with tempfile.TemporaryDirectory() as td:
        fat = os.path.join(td, "fat.bin")
        subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", LIB,
                        os.path.join(td, "junk")], check=True)
        data = open(fat, "rb").read()
        offs = [m.start() for m in re.finditer(re.escape(MAGIC), data)]
        for k, a in enumerate(offs):
            b = offs[k + 1] if k + 1 < len(offs) else len(data)
            part, co = os.path.join(td, f"b{k}.bin"), os.path.join(td, f"b{k}.co")
            open(part, "wb").write(data[a:b])
            r = subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o",
                                "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--input={part}",
                                f"--output={co}"], capture_output=True)
            if r.returncode or not os.path.exists(co) or os.path.getsize(co) == 0:
                continue
            notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], capture_output=True,
                                   text=True).stdout
            for blk in notes.split("  - .agpr_count")[1:]:
                def get(key):
                    m = re.search(rf"\.{key}:\s+(\S+)", blk)
                    return m.group(1) if m else None
                out[get("name")] = {"private": int(get("private_segment_fixed_size") or 0),
                                    "dynamic_stack": get("uses_dynamic_stack") == "true",
                                    "vgpr": int(get("vgpr_count") or 0)}
    return out


def test_box_marches_use_no_scratch():
    ks = _kernels()
    box = {n: v for n, v in ks.items() if n and re.match(r"_ZN2vr(11k_march_duo|7k_march)I", n)}
    duo = [n for n in box if "k_march_duo" in n]
    # every (B, M, K) instance of the duo ships: B in 1, 2, 4, 8; M in 1, 2; K in 2..4
    assert len(duo) == 4 * 2 * 3, sorted(duo)
    plain = [n for n in box if "k_march_duo" not in n]
    assert plain, "no k_march instance in libvr.so"
    bad = {n: v for n, v in box.items() if v["private"] or v["dynamic_stack"]}
    assert not bad, bad
    assert all(v["vgpr"] <= 256 for v in box.values()), {n: v["vgpr"] for n, v in box.items()}
