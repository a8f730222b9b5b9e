"""Canonical numerics of the oracle: accuracy against float64 libm."""
import numpy as np

from oracle import oracle as O


def _ulp_err(got, ref):
    ref32 = np.abs(ref).astype(np.float32)
    return np.abs(got.astype(np.float64) - ref) / np.spacing(np.maximum(ref32, np.float32(1e-30)))


def test_tanh_accuracy():
    xs = np.linspace(-12, 12, 40001).astype(np.float32)
    f = O.math_fn("tanh")
    got = np.array([f(float(x)) for x in xs], np.float32)
    assert _ulp_err(got, np.tanh(xs.astype(np.float64))).max() < 6


def test_exp_accuracy():
    xs = np.linspace(-87, 88, 40001).astype(np.float32)
    f = O.math_fn("exp")
    got = np.array([f(float(x)) for x in xs], np.float32)
    assert _ulp_err(got, np.exp(xs.astype(np.float64))).max() < 2
    assert f(0.0) == 1.0 and f(-200.0) == 0.0


def test_exp64_matches_numpy_after_f32_cast():
    x = -np.random.default_rng(0).uniform(0, 800, 100000)
    f = O.math_fn("exp64")
    got = np.array([f(float(v)) for v in x])
    assert np.array_equal(got.astype(np.float32), np.exp(x).astype(np.float32))
    assert np.max(np.abs(got - np.exp(x)) / np.maximum(np.exp(x), 1e-300)) < 5e-16


def test_gelu_matches_jax_formula():
    xs = np.linspace(-8, 8, 20001).astype(np.float32)
    f = O.math_fn("gelu")
    got = np.array([f(float(x)) for x in xs], np.float32)
    x = xs.astype(np.float64)
    ref = x * 0.5 * (1 + np.tanh(np.sqrt(2 / np.pi) * (x + 0.044715 * x ** 3)))
    assert np.abs(got - ref).max() < 2e-6


def test_doubled_gelu_identity(tmp_path):
    """The encoder kernels evaluate 2·GELU(x) as x + x·tanh(u) (one fma less than h + h·tanh(u))
    and feed it to weights pre-scaled by 0.5 (pst_device.h c_gelu2x, pst_api.cpp): exact iff
    fma(x, t, x) == 2·fma(x/2, t, x/2) bitwise. tools/micro/gelu_double_check.c checks every
    float32 input (no mismatch for |x| >= 2^-125); here every 101st input."""
    import os
    import subprocess
    src = os.path.join(os.path.dirname(__file__), "..", "tools", "micro", "gelu_double_check.c")
    exe = str(tmp_path / "gdc")
    subprocess.run(["gcc", "-O2", "-fopenmp", "-mfma", "-DSTRIDE=101", src, "-o", exe, "-lm"], check=True)
    out = subprocess.run([exe], capture_output=True, text=True, env=dict(os.environ, OMP_NUM_THREADS="4"))
    assert out.returncode == 0, out.stdout + out.stderr
    assert " 0 mismatches with |x| >= 2^-125" in out.stdout, out.stdout
