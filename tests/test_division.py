"""The march divides by the reference's constants with a reciprocal multiply and
one FMA correction (vr_device.h div_const).  tests/c/divcheck.c proves, over all
2^32 float inputs, that this is bit-identical to the reference's double division
(K:758, 759, 766), and that the float-only variance division (div_var_f32) and the
multiply-only form for float results (div_to_float) are too, and so is the
entropy's split-reciprocal division by ln 2 (div_ln2).  CPU only (gcc + OpenMP, ~15 s on 8 cores)."""
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))


def test_fast_division_is_exact_for_every_float(tmp_path):
    exe = tmp_path / "divcheck"
    subprocess.run(["gcc", "-O2", "-fopenmp", "-ffp-contract=off",
                    os.path.join(HERE, "c", "divcheck.c"), "-o", str(exe), "-lm"], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.count("mismatches: 0") == 7, r.stdout
