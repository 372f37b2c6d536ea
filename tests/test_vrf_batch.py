"""The eight-lane AVX-512 IFMA VRF outputs (csrc/runtime/vrf_ifma.cpp) against the scalar path (vrf.cpp): the
noiser lottery consumes these bytes, so the batch must be byte-identical for every key, alpha and batch size.
On a CPU without IFMA vrf_beta_batch falls back to the scalar code and the tests check that path instead."""
import os
import random
import subprocess
import sys

from biscotti_amd.native import rt


def _seeds(n, seed=0):
    r = random.Random(seed)
    return [bytes(r.getrandbits(8) for _ in range(32)) for _ in range(n)]


def test_batch_outputs_match_scalar_every_batch_size():
    R = rt()
    seeds = _seeds(33)
    r = random.Random(1)
    for n in list(range(1, 18)) + [33]:
        alpha = bytes(r.getrandbits(8) for _ in range(r.choice([0, 7, 32, 45])))
        assert R.vrf_beta_batch(seeds[:n], alpha) == [R.vrf_beta(s, alpha) for s in seeds[:n]], n


def test_batch_outputs_many_alphas():
    """Many (key, alpha) pairs: every lane takes its own number of encode_to_curve attempts."""
    R = rt()
    seeds = _seeds(8, seed=2)
    for k in range(40):
        alpha = k.to_bytes(4, "little") * 8
        assert R.vrf_beta_batch(seeds, alpha) == [R.vrf_beta(s, alpha) for s in seeds]


def test_outputs_only_job_uses_the_batch_and_matches():
    """The round's VRF job (outputs only, the device makes the proofs) with enough outputs per thread takes the
    batch path; the same job with BISCOTTI_VRF_SCALAR set (scalar path) gives the same bytes."""
    code = ("import sys; from biscotti_amd.native import rt; R = rt(); "
            "seeds = [bytes([i]) * 32 for i in range(1, 41)]; "
            "j = R.vrf_prove_batch_async(seeds, b'block hash', 2, None, True); "
            "out = [b.hex() for b, _ in j.result()]; "
            "assert out == [R.vrf_beta(s, b'block hash').hex() for s in seeds]; print(out[0], out[-1])")
    got = []
    for scalar in (False, True):
        env = dict(os.environ)
        env.pop("BISCOTTI_VRF_SCALAR", None)
        if scalar:
            env["BISCOTTI_VRF_SCALAR"] = "1"
        p = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120)
        assert p.returncode == 0, p.stderr
        got.append(p.stdout.strip())
    assert got[0] == got[1]


def test_batch_proofs_match_scalar_and_verify():
    """vrf_prove_batch (outputs + proofs, eight keys per IFMA batch: encode_to_curve, x*H, k*H, the fixed-base
    k*B and the three encodings with one inversion) is byte-identical to vrf_prove and verifies; also through
    the job that proves the run's last round on the host (vrf_proofs_async)."""
    R = rt()
    seeds = _seeds(19, seed=3)
    for alpha in (b"", b"block hash", bytes(range(40))):
        got = R.vrf_prove_batch_ifma(seeds, alpha)
        ref = [R.vrf_prove_batch_async([s], alpha, 1).result()[0] for s in seeds]
        assert got == ref
        assert R.vrf_proofs_async(seeds, alpha, 3).result() == ref
        for s, (beta, pi) in zip(seeds, got):
            assert R.vrf_verify(R.ed25519_public_key(s), alpha, pi) == beta
