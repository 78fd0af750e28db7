"""The entropy's exact float logarithm (vr_device.h logf_fast_tabp, K:766's
logf) restated on the host with the generated table (csrc/vr_logtab.h,
tools/gen_logtab.py): equal to (float)log((double)x) wherever it claims
exactness, for every positive finite float, and leaving fewer than 2^16 inputs
to the double log.  CPU only (g++ + OpenMP, a few seconds on 8 cores); the
device code itself is checked the same way by test_fast_log_is_exact_for_every_float
(tests/test_gpu_parity.py)."""
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(os.path.dirname(HERE), "volume-rendering-based-on-distribution-data_amd", "csrc")


def test_fast_log_restatement_is_exact_for_every_float(tmp_path):
    exe = tmp_path / "logcheck"
    subprocess.run(["g++", "-O2", "-fopenmp", "-ffp-contract=off", "-I", CSRC,
                    os.path.join(HERE, "c", "logcheck.cpp"), "-o", str(exe)], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "fast-form mismatches: 0" in r.stdout, r.stdout
