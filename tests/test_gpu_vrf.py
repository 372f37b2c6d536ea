"""Device ECVRF prover (kernels/vrf.hip) bit-exact against the host runtime (RFC 9381 pinned in
test_crypto.py::test_ecvrf_rfc9381_vector): proofs, outputs, verification, round-batched queue."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_device_vrf_proofs_match_host(rt):
    from biscotti_amd.ops.vrf import DeviceVrfProver
    prover = DeviceVrfProver("cuda")
    rng = np.random.default_rng(3)
    seeds = [bytes(rng.integers(0, 256, 32, dtype=np.uint8)) for _ in range(150)]
    alphas = [os.urandom(32), bytes(32), b"\xff" * 32]
    al = [alphas[i % 3] for i in range(len(seeds))]
    pi, beta = prover.prove(seeds, al, beta=True)
    torch.cuda.synchronize()
    pi, beta = pi.cpu().numpy(), beta.cpu().numpy()
    for i, (s, a) in enumerate(zip(seeds, al)):
        hb, hp = rt.vrf_prove(s, a)
        assert bytes(pi[i]) == hp, i
        assert bytes(beta[i]) == hb, i
        assert rt.vrf_beta(s, a) == hb
    assert rt.vrf_verify(rt.vrf_public_key(seeds[0]), al[0], bytes(pi[0])) == bytes(beta[0])


def test_outputs_only_job_and_device_queue(rt):
    from biscotti_amd.ops.vrf import DeviceVrfProver
    seeds = [os.urandom(32) for _ in range(40)]
    alpha = os.urandom(32)
    job = rt.vrf_prove_batch_async(seeds, alpha, 4, None, True)
    full = rt.vrf_prove_batch(seeds, alpha, 4)
    assert job.betas() == [b for b, _ in full]
    prover = DeviceVrfProver("cuda", batch_rounds=2)
    st = torch.cuda.Stream()
    prover.submit(seeds[:20], alpha, st)
    assert prover.proofs == 0
    prover.submit(seeds[20:], alpha, st)       # second round: one launch for both
    assert prover.proofs == 40
    prover.submit(seeds[:5], alpha, st)
    prover.drain(st)
    assert prover.proofs == 45
