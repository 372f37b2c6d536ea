"""Key bootstrap tool: ``python -m biscotti_amd.keygen -n <nodes per host> -d <dimensions> [-h hosts] [-o dir]``.

Equivalent of keyGeneration/generateBootstrapFile.go:43-207:
  * ``commitKey.json`` -- d JSON lines ``{"Id":i,"Pkey":<G1 64 B>,"Skey":<G2 129 B>}`` with
    PK_G1[i] = s^i G1 and PK_G2[i] = s^i G2, s = 2 (publicKey.go:26-61, s hard-coded at :36);
  * ``pKeyG1.json`` -- one ``{"Id":i,"Pkey":<G1 64 B>,"Skey":<scalar 32 B BE>}`` line per peer with a
    fresh Schnorr keypair (publicKey.go:81-99);
  * ``peersfile.txt`` -- ``host:port`` per peer, ports 8000 + i counted across all hosts, ``-n`` peers
    per line of the hosts file (generateBootstrapFile.go:141-156).
Byte layouts are kyber's marshals (base64 in JSON, Go's []byte encoding), written by the native
runtime.  Without ``-h`` a single host 127.0.0.1 is used (the localTest.sh layout).
"""
from __future__ import annotations

import argparse
import os
import secrets
import sys


def generate(out_dir: str, nodes_per_host: int, dims: int, hosts: list[str] | None = None,
             secret: int = 2, entropy_seed: bytes | None = None) -> dict:
    """Write the three bootstrap files; returns their paths.  `entropy_seed` makes the client keys
    reproducible (tests); by default they come from the OS CSPRNG like GenerateClientKey."""
    import hashlib

    from .native import rt

    R = rt()
    hosts = hosts or ["127.0.0.1"]
    os.makedirs(out_dir, exist_ok=True)
    paths = {"commit_key": os.path.join(out_dir, "commitKey.json"),
             "pkey_g1": os.path.join(out_dir, "pKeyG1.json"),
             "peers": os.path.join(out_dir, "peersfile.txt")}
    R.write_commit_key(paths["commit_key"], dims, secret)
    keys, lines = [], []
    i = 0
    for h in hosts:
        for _ in range(nodes_per_host):
            lines.append(f"{h}:{8000 + i}")
            ent = hashlib.sha256(entropy_seed + i.to_bytes(8, "little")).digest() if entropy_seed else \
                secrets.token_bytes(32)
            keys.append(R.client_key_from_entropy(ent))
            i += 1
    R.write_client_keys(paths["pkey_g1"], keys)
    with open(paths["peers"], "w") as f:
        f.write("".join(ln + "\n" for ln in lines))
    return paths


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="biscotti_amd.keygen", description=__doc__, add_help=False,
                                 formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--help", action="help")
    ap.add_argument("-n", dest="nodes", type=int, default=0, help="nodes per host")
    ap.add_argument("-d", dest="dims", type=int, default=0, help="number of model parameters")
    ap.add_argument("-h", dest="hosts", default=None, help="hosts file (one hostname / IP per line)")
    ap.add_argument("-o", dest="out", default=".", help="output directory")
    ap.add_argument("--secret", type=int, default=2, help="commitment-key secret s (reference: 2)")
    ns = ap.parse_args(argv)
    if ns.nodes <= 0 or ns.dims <= 0:
        ap.print_usage()
        return 1
    hosts = None
    if ns.hosts:
        with open(ns.hosts) as f:
            hosts = [ln.strip() for ln in f if ln.strip()]
    paths = generate(ns.out, ns.nodes, ns.dims, hosts, ns.secret)
    print(ns.nodes * len(hosts or [1]))
    print("Done writing", *paths.values())
    return 0


if __name__ == "__main__":
    sys.exit(main())
