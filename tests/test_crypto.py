"""BN256 / Schnorr / hashing / VRF tests of the native host runtime.

Golden vectors: the reference's binary key files (tests/fixtures, copied from
/root/reference/keyGeneration): kyber-produced G1/G2 marshals and (sk, pk = sk*G) pairs.
"""
import hashlib
import random

import pytest


def _records(path, size):
    data = path.read_bytes()
    step = size + 1
    assert len(data) % step == 0
    return [data[i:i + size] for i in range(0, len(data), step)]


def test_prime_and_order(rt):
    u = 6518589491078791937
    assert rt.bn256_prime() == 36 * u**4 + 36 * u**3 + 24 * u**2 + 6 * u + 1
    assert rt.bn256_order() == 36 * u**4 + 36 * u**3 + 18 * u**2 + 6 * u + 1


def test_generator_marshal_matches_kyber(rt, fixtures):
    g1 = _records(fixtures / "commitKeyG1", 64)
    assert g1[0] == rt.g1_generator()
    p = rt.bn256_prime()
    assert int.from_bytes(g1[0][:32], "big") == 1 and int.from_bytes(g1[0][32:], "big") == p - 2
    g2 = _records(fixtures / "commitKeyG2", 129)
    assert g2[0] == rt.g2_generator()


def test_kyber_points_decode(rt, fixtures):
    for rec in _records(fixtures / "commitKeyG1", 64):
        assert rt.g1_is_valid(rec)
    for rec in _records(fixtures / "commitKeyG2", 129):
        assert rt.g2_is_valid(rec)
    bad = bytearray(_records(fixtures / "commitKeyG1", 64)[3])
    bad[63] ^= 1
    assert not rt.g1_is_valid(bytes(bad))


def test_client_keys_sk_times_g(rt, fixtures):
    pks = _records(fixtures / "pKeyG1", 64)
    sks = _records(fixtures / "sKeyG1", 32)
    gen = rt.g1_generator()
    for sk, pk in zip(sks, pks):
        s = int.from_bytes(sk, "big")
        assert rt.g1_mul(gen, s) == pk
        assert rt.g1_base_mul(s) == pk


def test_group_laws(rt):
    g = rt.g1_generator()
    order = rt.bn256_order()
    assert rt.g1_mul(g, order) == rt.g1_infinity()
    a, b = 123456789, 987654321
    assert rt.g1_add(rt.g1_mul(g, a), rt.g1_mul(g, b)) == rt.g1_mul(g, a + b)
    # doubling path inside add, and P + (-P)
    p = rt.g1_mul(g, 77)
    assert rt.g1_add(p, p) == rt.g1_mul(g, 154)
    assert rt.g1_add(p, rt.g1_neg(p)) == rt.g1_infinity()
    # negative scalar == (Order - |k|) * P (kyber SetInt64 semantics)
    assert rt.g1_mul_i64(p, -5) == rt.g1_mul(p, order - 5)
    g2 = rt.g2_generator()
    assert rt.g2_mul(g2, order) == b"\x00"
    assert rt.g2_add(rt.g2_mul(g2, 2), rt.g2_mul(g2, 4)) == rt.g2_mul(g2, 6)


def test_scalar_marshal(rt):
    order = rt.bn256_order()
    assert int.from_bytes(rt.scalar_from_i64(-1), "big") == order - 1
    assert int.from_bytes(rt.scalar_from_i64(7), "big") == 7


def test_schnorr_roundtrip(rt):
    sk, pk = rt.client_key_from_entropy(b"peer-7")
    msg = rt.g1_mul(rt.g1_generator(), 4242)  # commitments are what verifiers sign
    sig = rt.schnorr_sign(msg, sk, b"nonce-entropy")
    assert len(sig) == 64
    assert rt.schnorr_verify(msg, pk, sig)
    assert not rt.schnorr_verify(msg[:-1] + bytes([msg[-1] ^ 1]), pk, sig)
    sk2, pk2 = rt.client_key_from_entropy(b"peer-8")
    assert not rt.schnorr_verify(msg, pk2, sig)
    batch = rt.schnorr_sign_batch([msg, msg[::-1]], sk, [b"a", b"b"], 2)
    assert rt.schnorr_verify(msg, pk, batch[0]) and rt.schnorr_verify(msg[::-1], pk, batch[1])


def test_sha_and_blake2b_against_hashlib(rt):
    rnd = random.Random(1)
    for n in [0, 1, 55, 56, 63, 64, 65, 111, 112, 127, 128, 129, 1000]:
        d = bytes(rnd.getrandbits(8) for _ in range(n))
        assert rt.sha256(d) == hashlib.sha256(d).digest()
        assert rt.sha512(d) == hashlib.sha512(d).digest()
        assert rt.blake2b(d, 64, b"") == hashlib.blake2b(d).digest()
        assert rt.blake2b(d, 20, b"k" * 64) == hashlib.blake2b(d, digest_size=20, key=b"k" * 64).digest()


def _blake2b_param_py(param: bytes, data: bytes) -> bytes:
    """Independent pure-Python BLAKE2b (RFC 7693) with an explicit parameter block."""
    M = (1 << 64) - 1
    IV = [0x6A09E667F3BCC908, 0xBB67AE8584CAA73B, 0x3C6EF372FE94F82B, 0xA54FF53A5F1D36F1,
          0x510E527FADE682D1, 0x9B05688C2B3E6C1F, 0x1F83D9ABFB41BD6B, 0x5BE0CD19137E2179]
    S = [[0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15], [14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3],
         [11, 8, 12, 0, 5, 2, 15, 13, 10, 14, 3, 6, 7, 1, 9, 4], [7, 9, 3, 1, 13, 12, 11, 14, 2, 6, 5, 10, 4, 0, 15, 8],
         [9, 0, 5, 7, 2, 4, 10, 15, 14, 1, 11, 12, 6, 8, 3, 13], [2, 12, 6, 10, 0, 11, 8, 3, 4, 13, 7, 5, 15, 14, 1, 9],
         [12, 5, 1, 15, 14, 13, 4, 10, 0, 7, 6, 3, 9, 2, 8, 11], [13, 11, 7, 14, 12, 1, 3, 9, 5, 0, 15, 4, 8, 6, 2, 10],
         [6, 15, 14, 9, 11, 3, 0, 8, 12, 2, 13, 7, 1, 4, 10, 5], [10, 2, 8, 4, 7, 6, 1, 5, 15, 11, 9, 14, 3, 12, 13, 0]]
    rot = lambda x, n: ((x >> n) | (x << (64 - n))) & M
    h = [IV[i] ^ int.from_bytes(param[8 * i:8 * i + 8], "little") for i in range(8)]
    outlen = param[0]
    blocks = [data[i:i + 128] for i in range(0, len(data), 128)] or [b""]
    t = 0
    for bi, blk in enumerate(blocks):
        last = bi == len(blocks) - 1
        t += len(blk)
        blk = blk.ljust(128, b"\0")
        m = [int.from_bytes(blk[8 * i:8 * i + 8], "little") for i in range(16)]
        v = h + IV
        v[12] ^= t & M
        v[13] ^= t >> 64
        if last:
            v[14] ^= M
        for r in range(12):
            s = S[r % 10]
            for (a, b, c, d), (x, y) in zip([(0, 4, 8, 12), (1, 5, 9, 13), (2, 6, 10, 14), (3, 7, 11, 15),
                                              (0, 5, 10, 15), (1, 6, 11, 12), (2, 7, 8, 13), (3, 4, 9, 14)],
                                             [(s[2 * i], s[2 * i + 1]) for i in range(8)]):
                v[a] = (v[a] + v[b] + m[x]) & M; v[d] = rot(v[d] ^ v[a], 32)
                v[c] = (v[c] + v[d]) & M; v[b] = rot(v[b] ^ v[c], 24)
                v[a] = (v[a] + v[b] + m[y]) & M; v[d] = rot(v[d] ^ v[a], 16)
                v[c] = (v[c] + v[d]) & M; v[b] = rot(v[b] ^ v[c], 63)
        h = [h[i] ^ v[i] ^ v[i + 8] for i in range(8)]
    return b"".join(x.to_bytes(8, "little") for x in h)[:outlen]


def test_blake2xb_structure(rt):
    """blake2xb (kyber XOF) = BLAKE2X over BLAKE2b: keyed root with xof-length 2^32-1, then
    output nodes B2(leaf=64, node_offset=i, inner=64) of the root digest."""
    seed, msg = bytes(range(64)), b"commitment-bytes"
    root = hashlib.blake2b(msg, digest_size=64, key=seed, node_offset=0xFFFFFFFF << 32).digest()
    out = rt.blake2xb(seed, msg, 200)
    expect = b""
    for i in range(4):
        p = bytearray(64)
        p[0] = 64
        p[4] = 64
        p[8:12] = i.to_bytes(4, "little")
        p[12:16] = b"\xff\xff\xff\xff"
        p[17] = 64
        assert rt.blake2b_param(bytes(p), root) == _blake2b_param_py(bytes(p), root)
        expect += _blake2b_param_py(bytes(p), root)
    assert out == expect[:200]
    # seeds longer than 64 bytes: tail is absorbed as message prefix
    long_seed = bytes(range(100))
    root2 = hashlib.blake2b(long_seed[64:] + msg, digest_size=64, key=long_seed[:64],
                            node_offset=0xFFFFFFFF << 32).digest()
    p = bytearray(64); p[0] = 64; p[4] = 64; p[12:16] = b"\xff" * 4; p[17] = 64
    assert rt.blake2xb(long_seed, msg, 64) == _blake2b_param_py(bytes(p), root2)


def test_ed25519_rfc8032_vector(rt):
    seed = bytes.fromhex("9d61b19deffd5a60ba844af492ec2cc44449c5697b326919703bac031cae7f60")
    assert rt.ed25519_public_key(seed).hex() == "d75a980182b10ab7d54bfed3c964073a0ee172f3daa62325af021a68f707511a"


def test_vrf_properties(rt):
    seed = bytes(range(32))
    pk = rt.vrf_public_key(seed)
    beta, pi = rt.vrf_prove(seed, b"block-hash")
    assert len(beta) == 64 and len(pi) == 80
    assert rt.vrf_verify(pk, b"block-hash", pi) == beta
    assert rt.vrf_prove(seed, b"block-hash") == (beta, pi)  # deterministic
    assert rt.vrf_verify(pk, b"block-hasH", pi) is None
    bad = bytearray(pi); bad[40] ^= 1
    assert rt.vrf_verify(pk, b"block-hash", bytes(bad)) is None
    other = rt.vrf_prove(bytes(32), b"block-hash")[0]
    assert other != beta
    batch = rt.vrf_prove_batch([seed, bytes(32)], b"block-hash", 2)
    assert batch[0] == (beta, pi) and batch[1][0] == other


def test_marshal_jac_batch_matches_single(rt):
    """Batch normalisation (one inversion via Montgomery's trick) == per-point marshal, incl. infinity."""
    import random

    import numpy as np

    p = 65000549695646603732796438742359905742825358107623003571877145026864184071783
    R = 1 << 256
    rng = random.Random(5)
    rows, want = [], []
    for k in [3, 17, 1 << 40, 99991, 5]:
        m = rt.g1_base_mul(k)
        aff = np.asarray(rt.g1_affine_mont_u32(m), dtype=np.uint32).reshape(-1)
        to_int = lambda a: sum(int(v) << (32 * i) for i, v in enumerate(a))
        xm, ym = to_int(aff[:8]), to_int(aff[8:16])
        z = rng.randrange(1, p)
        x, y = xm * pow(R, -1, p) % p, ym * pow(R, -1, p) % p
        X, Y = x * z * z % p, y * z * z * z % p
        limbs = lambda v: [(v * R % p >> (32 * i)) & 0xFFFFFFFF for i in range(8)]
        rows.append(limbs(X) + limbs(Y) + limbs(z))
        want.append(m)
    rows.insert(2, [0] * 24)  # point at infinity (z == 0)
    want.insert(2, rt.g1_infinity())
    got = rt.g1_marshal_jac_batch(np.asarray(rows, dtype=np.uint32))
    assert got.shape == (6, 64)
    for g, w in zip(got, want):
        assert bytes(g) == (w if len(w) == 64 else bytes(64))
    single = rt.g1_marshal_jac_u32(np.asarray(rows, dtype=np.uint32))
    assert [bytes(g) for g in got] == [s if len(s) == 64 else bytes(64) for s in single]


def test_ecvrf_rfc9381_vector(rt):
    """RFC 9381 ECVRF-EDWARDS25519-SHA512-TAI example (SK = RFC 8032 test 1, alpha = empty)."""
    seed = bytes.fromhex("9d61b19deffd5a60ba844af492ec2cc44449c5697b326919703bac031cae7f60")
    beta, pi = rt.vrf_prove(seed, b"")
    assert pi.hex() == ("8657106690b5526245a92b003bb079ccd1a92130477671f6fc01ad16f26f723f26f8a57ccaed74ee1b190b"
                        "ed1f479d9727d2d0f9b005a6e456a35d4fb0daab1268a1b0db10836d9826a528ca76567805")
    assert beta.hex() == ("90cf1df3b703cce59e2a35b925d411164068269d7b2d29f3301c03dd757876ff66b71dda49d2de59d0345"
                          "0451af026798e8f81cd2e333de5cdf4f3e140fdd8ae")
    assert rt.vrf_verify(rt.vrf_public_key(seed), b"", pi) == beta
    # batched prover (thread pool + key cache) agrees
    assert rt.vrf_prove_batch([seed] * 3, b"", 3) == [(beta, pi)] * 3


def test_vrf_async_jobs_match_sync(rt):
    import os

    seeds = [os.urandom(32) for _ in range(20)]
    j1 = rt.vrf_prove_batch_async(seeds, b"alpha", 4)
    j2 = rt.vrf_prove_batch_async(seeds[:5], b"beta", 4, j1)  # chained: starts after j1
    assert j2.result() == rt.vrf_prove_batch(seeds[:5], b"beta", 1)
    assert j1.done() and j1.result() == rt.vrf_prove_batch(seeds, b"alpha", 3)
    assert rt.vrf_prove_batch_async([], b"x", 4).result() == []


def test_schnorr_sign_multi_batch(rt):
    """Round-wide batched signing: per-message keys, derived nonces, one shared inversion."""
    import os

    keys = [rt.client_key_from_entropy(os.urandom(32)) for _ in range(3)]
    msgs = [os.urandom(64) for _ in range(25)]
    key_of = [i % 3 for i in range(25)]
    bases = [os.urandom(32) for _ in range(3)]
    ids = list(range(100, 125))
    sigs = rt.schnorr_sign_multi(msgs, [k[0] for k in keys], key_of, bases, ids, 4)
    for m, k, s in zip(msgs, key_of, sigs):
        assert rt.schnorr_verify(m, keys[k][1], s)
        assert not rt.schnorr_verify(m, keys[(k + 1) % 3][1], s)
    # deterministic, and equal to the single-signature path with the same nonce entropy
    assert rt.schnorr_sign_multi(msgs, [k[0] for k in keys], key_of, bases, ids, 1) == sigs
    ent = bases[key_of[7]] + (107).to_bytes(4, "little")
    assert rt.schnorr_sign(msgs[7], keys[key_of[7]][0], ent) == sigs[7]


def test_schnorr_sign_rows_matches_message_list(rt):
    """Table-row signing (messages = rows of a uint8 [n, 64] table) equals the list API, and the
    array result equals the bytes result."""
    import os

    import numpy as np

    keys = [rt.client_key_from_entropy(os.urandom(32)) for _ in range(2)]
    table = np.frombuffer(os.urandom(64 * 12), np.uint8).reshape(12, 64)
    rows = [5, 0, 11, 5, 3]
    key_of = [0, 1, 1, 0, 1]
    bases = [os.urandom(32) for _ in range(2)]
    ids = [7, 8, 9, 10, 11]
    want = rt.schnorr_sign_multi([table[r].tobytes() for r in rows], [k[0] for k in keys], key_of, bases, ids, 2)
    job = rt.schnorr_sign_rows_async(table, rows, [k[0] for k in keys], key_of, bases, ids, 3)
    arr = job.result_array()
    assert arr.shape == (5, 64) and [a.tobytes() for a in arr] == want
    with pytest.raises(RuntimeError):
        rt.schnorr_sign_rows_async(table, [12], [keys[0][0]], [0], bases[:1], [1], 1).result_array()


def test_schnorr_sign_rows_jac_matches_marshalled_rows(rt):
    """Signing device-layout Jacobian commitment rows (marshalled on the job's thread: the deferred verifier
    signatures) equals signing their marshals."""
    import os

    import numpy as np

    one = np.array([0xa1f76999, 0xe7a35393, 0xdf4a4a61, 0x11a4772e, 0x9e7b23de, 0x55901347, 0xb55c7806, 0x704afe1c],
                   np.uint32)   # Montgomery 1: an affine point's Z in Jacobian form
    pts = [rt.g1_base_mul(3 + 101 * k) for k in range(8)]
    jac = np.stack([np.concatenate([np.asarray(rt.g1_affine_mont_u32(p), np.uint32).reshape(-1)[:16], one])
                    for p in pts])
    table = rt.g1_marshal_jac_batch(jac)
    keys = [rt.client_key_from_entropy(os.urandom(32)) for _ in range(2)]
    rows, key_of, ids = [4, 0, 7, 4], [1, 0, 1, 0], [3, 4, 5, 6]
    bases = [os.urandom(32) for _ in range(2)]
    want = rt.schnorr_sign_rows_async(table, rows, [k[0] for k in keys], key_of, bases, ids, 2).result_array()
    got = rt.schnorr_sign_rows_jac_async(jac, rows, [k[0] for k in keys], key_of, bases, ids, 2).result_array()
    assert np.array_equal(got, want)
    with pytest.raises(RuntimeError):
        rt.schnorr_sign_rows_jac_async(jac, [8], [keys[0][0]], [0], bases[:1], [1], 1)


def test_concurrent_native_jobs_share_the_pool(rt):
    """VRF and signing jobs running at once (and a foreground batch) give the serial results."""
    import os

    seeds = [os.urandom(32) for _ in range(40)]
    import numpy as np

    keys = [rt.client_key_from_entropy(os.urandom(32)) for _ in range(2)]
    msgs = [os.urandom(64) for _ in range(60)]
    key_of = [i % 2 for i in range(60)]
    bases = [os.urandom(32), os.urandom(32)]
    ids = list(range(60))
    v = rt.vrf_prove_batch_async(seeds, b"h", 3)
    s = rt.schnorr_sign_multi_async(msgs, [k[0] for k in keys], key_of, bases, ids, 8)
    fg = rt.vrf_prove_batch(seeds[:10], b"g", 8)
    assert s.result() == rt.schnorr_sign_multi(msgs, [k[0] for k in keys], key_of, bases, ids, 1)
    assert v.result() == rt.vrf_prove_batch(seeds, b"h", 1)
    assert fg == rt.vrf_prove_batch(seeds[:10], b"g", 1)


def test_pairing_bilinear_and_kzg_witnesses(rt):
    """Optimal ate pairing (K13) + verifySecret (kyber.go:650-673) on our Shamir witnesses."""
    import random

    import numpy as np

    n = 65000549695646603732796438742359905742570406053903786389881062969044166799969
    g1, g2 = rt.g1_generator(), rt.g2_generator()
    one = rt.pairing_digest(g1, g2, 0)
    assert rt.pairing_digest(g1, g2) != one and rt.pairing_digest(g1, g2, n) == one
    rnd = random.Random(3)
    a, b = rnd.randrange(1, n), rnd.randrange(1, n)
    assert rt.pairing_digest(rt.g1_mul(g1, a), rt.g2_mul(g2, b)) == rt.pairing_digest(g1, g2, a * b % n)
    # KZG evaluation proofs of the secret shares
    s = 2
    key = rt.CommitKey.generate(25, s)
    coeffs = np.random.default_rng(0).integers(-10**6, 10**6, size=25)
    _, chunk_commits, ys, wits = key.make_shares(coeffs, 10, 21)
    g2s = rt.g2_mul(g2, s)
    for k, t in [(0, 0), (1, 10), (2, 20), (2, 3)]:
        x, y = t - 10, int(ys[k, t])
        yb = rt.g1_mul(g1, s ** (10 * k))          # PK_G1[10k]: chunk k is committed on PK[10k..]
        assert rt.verify_secret(chunk_commits[k], wits[k * 21 + t], g2, g2s, x, y, yb)
        assert not rt.verify_secret(chunk_commits[k], wits[k * 21 + t], g2, g2s, x, y + 1, yb)
        assert not rt.verify_secret(chunk_commits[k], wits[k * 21 + (t + 1) % 21], g2, g2s, x, y, yb)
    # the reference's literal check (y base = G1) holds for chunk 0 only (quirk Q9)
    assert rt.verify_secret(chunk_commits[0], wits[4], g2, g2s, -6, int(ys[0, 4]))
    assert not rt.verify_secret(chunk_commits[1], wits[21 + 4], g2, g2s, -6, int(ys[1, 4]))
    xs = [t - 10 for t in range(21)]
    ok = rt.verify_secrets_batch([chunk_commits[1]] * 21, wits[21:42], g2, g2s, xs, [int(v) for v in ys[1]], 4,
                                 rt.g1_mul(g1, s ** 10))
    assert all(ok)


def test_vrf_two_phase_outputs_match_full_proofs(rt):
    """betas() returns once every output is known; the full results (beta, pi) agree with it and
    with the one-shot prover, and every proof verifies."""
    import os as _os
    seeds = [bytes([i]) * 32 for i in range(1, 20)]
    alpha = _os.urandom(32)
    job = rt.vrf_prove_batch_async(seeds, alpha, 4)
    betas = job.betas()
    full = job.result()
    assert betas == [b for b, _ in full]
    for s, (b, pi) in zip(seeds, full):
        assert (b, pi) == tuple(rt.vrf_prove(s, alpha))


def test_batched_kzg_check_host(rt):
    """K13 on the host: the u-chain final exponentiation equals the generic exponent; the random
    linear combination of every (chunk, point) verifySecret accepts exactly when each check does."""
    import numpy as np

    assert rt.final_exp_selftest(2, 11)
    s = 3
    key = rt.CommitKey.generate(35, s)
    coeffs = np.random.default_rng(5).integers(-10**5, 10**5, size=35)
    _, cc, ys, wits = key.make_shares(coeffs, 10, 21)
    g2 = rt.g2_generator()
    g2s = rt.g2_mul(g2, s)
    xs = [t - 10 for t in range(21)]
    bases = [key.point(10 * k) for k in range(len(cc))]
    pts = rt.kzg_rlc_host(cc, wits, ys.reshape(-1), xs, bases, 42, 2)
    assert rt.kzg_check(*pts, g2, g2s)
    bad = list(wits)
    bad[30] = wits[31]
    assert not rt.kzg_check(*rt.kzg_rlc_host(cc, bad, ys.reshape(-1), xs, bases, 42, 2), g2, g2s)
    y2 = ys.copy()
    y2[2, 7] -= 1
    assert not rt.kzg_check(*rt.kzg_rlc_host(cc, wits, y2.reshape(-1), xs, bases, 42, 2), g2, g2s)
    # literal form (y against G1): chunk 0 only
    assert rt.kzg_check(*rt.kzg_rlc_host(cc[:1], wits[:21], ys[:1].reshape(-1), xs, [rt.g1_generator()], 7, 1), g2, g2s)
    assert not rt.kzg_check(*rt.kzg_rlc_host(cc, wits, ys.reshape(-1), xs, [rt.g1_generator()], 7, 1), g2, g2s)
