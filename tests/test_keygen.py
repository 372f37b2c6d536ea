"""Bootstrap-file tool: formats, reproducibility, and that the engine consumes what it writes."""
import base64
import json


def test_keygen_files(tmp_path, rt):
    from biscotti_amd.keygen import generate

    hosts = ["10.0.0.1", "10.0.0.2"]
    paths = generate(str(tmp_path), 3, 40, hosts, entropy_seed=b"x")
    peers = open(paths["peers"]).read().splitlines()
    assert peers == ["10.0.0.1:8000", "10.0.0.1:8001", "10.0.0.1:8002",
                     "10.0.0.2:8003", "10.0.0.2:8004", "10.0.0.2:8005"]
    ck = [json.loads(ln) for ln in open(paths["commit_key"])]
    assert [r["Id"] for r in ck] == list(range(40))
    g = rt.g1_generator()
    for i in (0, 1, 5, 39):
        assert base64.b64decode(ck[i]["Pkey"]) == rt.g1_mul(g, 2 ** i)      # PK_G1[i] = 2^i G1
        assert len(base64.b64decode(ck[i]["Skey"])) == 129                 # G2 marshal
    pk = [json.loads(ln) for ln in open(paths["pkey_g1"])]
    assert len(pk) == 6
    for r in pk:
        sk = base64.b64decode(r["Skey"])
        assert rt.g1_mul(g, int.from_bytes(sk, "big")) == base64.b64decode(r["Pkey"])
    assert rt.read_client_keys(paths["pkey_g1"])[2] == rt.read_client_keys(paths["pkey_g1"])[2]
    again = generate(str(tmp_path / "b"), 3, 40, hosts, entropy_seed=b"x")
    assert open(again["pkey_g1"]).read() == open(paths["pkey_g1"]).read()


def test_engine_uses_generated_keys(tmp_path):
    from biscotti_amd.keygen import generate
    from biscotti_amd.protocol.config import RunConfig
    from biscotti_amd.protocol.engine import BiscottiEngine

    paths = generate(str(tmp_path), 5, 25, None, entropy_seed=b"y")
    cfg = RunConfig(num_nodes=5, dataset="creditcard", num_verifiers=1, num_miners=2, num_noisers=1,
                    device="cpu", commit_key=paths["commit_key"], pkey_file=paths["pkey_g1"],
                    peers_file=paths["peers"], deterministic_time=True)
    eng = BiscottiEngine(cfg)
    for _ in range(2):
        eng.run_round()
    ok, why = eng.fsm.chain.verify()
    assert ok, why
