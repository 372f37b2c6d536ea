"""Exact check of scripts/isa/fpmul_f64.hip's output: for every pair, the FIPS result == a b 2^-256 mod p and the
double-FMA result (signed 48-bit limbs, R = 2^288) == a b 2^-288 mod p.  Prints one JSON line."""
import json
import sys

import numpy as np

P = 65000549695646603732796438742359905742825358107623003571877145026864184071783
n = 1 << 20
raw = open(sys.argv[1] if len(sys.argv) > 1 else "fpmul_f64_check.bin", "rb").read()
u = np.frombuffer(raw[: 3 * n * 32], dtype=np.uint32).reshape(3, n, 8)
f = np.frombuffer(raw[3 * n * 32:], dtype=np.float64).reshape(n, 6)
W = [1 << (32 * k) for k in range(8)]
L = [1 << (48 * k) for k in range(6)]
i256, i288 = pow(2, -256, P), pow(2, -288, P)
bad_fips = bad_f64 = bad_range = 0
for i in range(n):
    a = sum(int(x) * w for x, w in zip(u[0, i], W))
    b = sum(int(x) * w for x, w in zip(u[1, i], W))
    r = sum(int(x) * w for x, w in zip(u[2, i], W))
    limbs = f[i]
    if not all(float(v).is_integer() for v in limbs):
        bad_f64 += 1
        continue
    o = sum(int(v) * w for v, w in zip(limbs, L))
    ab = a * b % P
    bad_fips += r != ab * i256 % P
    bad_f64 += o % P != ab * i288 % P
    bad_range += not (-2 * P < o < 2 * P)
print(json.dumps({"check": "f64fma_48x6 vs exact", "n": n, "fips_mismatches": bad_fips, "f64_mismatches": bad_f64,
                  "f64_out_of_range": bad_range}))
