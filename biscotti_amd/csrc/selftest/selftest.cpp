// Native self-test of the host runtime, built with AddressSanitizer + UBSan by
// ``python -m biscotti_amd._build --sanitize`` and with ThreadSanitizer by ``--tsan`` (host code only: GPU
// sanitizers are not used).  It drives every runtime module from several threads at once and checks known
// answers, and stresses the thread pool and job dispatcher the bindings run their batches on (overlapping
// jobs from several submitting threads, jobs that wait on earlier jobs), so memory errors, UB and data races
// that the Python tests cannot see show up here.
#include <atomic>
#include <cstdio>
#include <cstring>
#include <future>
#include <thread>
#include <vector>

#include "bn256.hpp"
#include "hash.hpp"
#include "keys.hpp"
#include "ledger.hpp"
#include "pairing.hpp"
#include "pool.hpp"
#include "protocol.hpp"
#include "shares.hpp"
#include "vrf.hpp"

using namespace bsc;

static std::atomic<int> failures{0};
#define CHECK(c)                                                        \
  do {                                                                  \
    if (!(c)) {                                                         \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      failures++;                                                       \
    }                                                                   \
  } while (0)

static void test_hash() {
  const Bytes abc = {'a', 'b', 'c'};
  CHECK(hex(Sha256::digest(abc)) == "ba7816bf8f01cfea414140de5dae2223b00361a396177a9cb410ff61f20015ad");
  Bytes big(100000);
  for (size_t i = 0; i < big.size(); ++i) big[i] = u8(i * 7);
  Sha256 inc;
  inc.update(big.data(), 333);
  inc.update(big.data() + 333, big.size() - 333);
  u8 a[32];
  inc.final(a);
  CHECK(Bytes(a, a + 32) == Sha256::digest(big));
  CHECK(hex(Sha512::digest(abc)).rfind("ddaf35a193617aba", 0) == 0);
}

static void test_curve() {
  const G1 g = G1::generator();
  const G1 a = g.mul_i64(123456789), b = g.mul_i64(-987654321);
  CHECK(a.add(b).equals(g.mul_i64(123456789 - 987654321)));
  CHECK(G1::unmarshal(a.marshal()).equals(a));
  CHECK(g.add(g.neg()).is_inf());
  const G2 h = G2::generator();
  CHECK(h.add(h).equals(h.dbl()));
  CHECK(G2::unmarshal(h.dbl().marshal()).equals(h.dbl()));
  const Scalar sk = Scalar::from_i64(424242);
  const G1 pk = g.mul(sk.v);
  const Bytes msg = {1, 2, 3, 4};
  const Bytes sig = schnorr_sign(msg, sk, Bytes(32, 7));
  CHECK(schnorr_verify(msg, pk, sig));
  CHECK(!schnorr_verify(Bytes{1, 2, 3, 5}, pk, sig));
}

static void test_pairing() {
  const G1 g = G1::generator();
  const G2 h = G2::generator();
  const Fp12 e = pairing(g, h);
  CHECK(!e.is_one());
  CHECK(pairing(g.mul_i64(6), h) == e.pow(U256::from_u64(6)));
}

static void test_vrf() {
  const Bytes seed = {0x9d, 0x61, 0xb1, 0x9d, 0xef, 0xfd, 0x5a, 0x60, 0xba, 0x84, 0x4a, 0xf4, 0x92, 0xec, 0x2c, 0xc4,
                      0x44, 0x49, 0xc5, 0x69, 0x7b, 0x32, 0x69, 0x19, 0x70, 0x3b, 0xac, 0x03, 0x1c, 0xae, 0x7f, 0x60};
  const auto out = vrf_prove(VrfKey::cached(seed), Bytes());
  CHECK(hex(out.second).rfind("8657106690b5526245a92b003bb079cc", 0) == 0);
  Bytes beta;
  CHECK(vrf_verify(VrfKey::cached(seed).pk, Bytes(), out.second, &beta) && beta == out.first);
}

static void test_shares_and_ledger() {
  const std::vector<G1> pk = gen_commit_key_g1(23, Scalar::from_i64(2));
  std::vector<i64> c(23);
  for (int i = 0; i < 23; ++i) c[size_t(i)] = (i * 7919) % 2001 - 1000;
  const SharePackage sp = make_shares(c, pk, 10, 21);
  CHECK(sp.commitment.equals(commit(c, pk, 0)));
  const std::vector<i64> xs = share_xs(21);
  for (int k = 0; k < 3; ++k) {
    std::vector<i64> ys(sp.ys.begin() + 21 * k, sp.ys.begin() + 21 * (k + 1)), got;
    CHECK(recover_exact(xs, ys, 9, &got));
    for (int j = 0; j < 10 && 10 * k + j < 23; ++j) CHECK(got[size_t(j)] == c[size_t(10 * k + j)]);
  }
  Blockchain chain = Blockchain::with_genesis(5);
  for (int it = 0; it < 3; ++it) {
    BlockData d;
    d.iteration = it;
    d.global_w = {0.5 * it, -1.25, 3.0, 1e-7, 2.0};
    Update u;
    u.iteration = it;
    u.commitment = sp.commitment.marshal();
    u.accepted = true;
    d.deltas.push_back(u);
    chain.append(chain.make_block(d, {{0, 10}, {1, 15}}, 1000 + it));
  }
  CHECK(chain.verify());
  CHECK(!chain.print_chain().empty());
}

static void test_protocol() {
  ProtocolConfig pc;
  pc.num_nodes = 30;
  pc.derive();
  std::map<i64, i64> stake;
  for (i64 i = 0; i < 30; ++i) stake[i] = 10 + 5 * (i % 4);
  std::vector<i64> v, m;
  select_roles(stake, Sha256::digest(Bytes{9}), 3, 3, 30, &v, &m);
  CHECK(v.size() == 3 && m.size() == 3);
  CHECK(select_noisers(stake, Sha256::digest(Bytes{8}), 4, 2, 30).size() == 2);
}

// The bindings' concurrency: several threads each run pool jobs (overlapping: the persistent workers help
// whichever job has items left) and submit dispatcher tasks that themselves run pool jobs and wait on a task
// submitted before them (the VrfJob::after / SignJob::after_vrf pattern).
static void test_pool(int t) {
  for (int rep = 0; rep < 4; ++rep) {
    const size_t n = 200 + 37 * size_t(t) + size_t(rep);
    std::vector<long long> out(n, 0);
    parallel_for(n, 4 + t % 3, [&](size_t i) { out[i] = (long long)(i * i) + t; });
    long long sum = 0;
    for (size_t i = 0; i < n; ++i) sum += out[i];
    long long want = 0;
    for (size_t i = 0; i < n; ++i) want += (long long)(i * i) + t;
    CHECK(sum == want);
  }
  std::promise<long long> first_p;
  std::shared_future<long long> first = first_p.get_future().share();
  std::promise<long long> second_p;
  std::future<long long> second = second_p.get_future();
  std::vector<long long> a(300, 0);
  dispatcher().submit([&] {
    parallel_for(a.size(), 3, [&](size_t i) { a[i] = (long long)i * 3; });
    long long s = 0;
    for (long long v : a) s += v;
    first_p.set_value(s);
  });
  dispatcher().submit([&, first] {
    const long long f = first.get();   // runs once the earlier task is done
    second_p.set_value(f + a[299]);
  });
  const long long got = second.get();
  CHECK(got == 3ll * 299 * 300 / 2 + 3ll * 299);
  CHECK(first.get() == 3ll * 299 * 300 / 2);
}

int main(int argc, char** argv) {
  if (argc > 1 && std::strcmp(argv[1], "pool") == 0) {
    // the concurrency stress alone (ThreadSanitizer runs: the crypto modules are ~10x slower under it)
    std::vector<std::thread> ts;
    for (int t = 0; t < 6; ++t) ts.emplace_back([t] { test_pool(t); test_hash(); test_protocol(); });
    for (auto& t : ts) t.join();
    std::printf("selftest pool: %s (%d failures)\n", failures ? "FAILED" : "ok", failures.load());
    return failures ? 1 : 0;
  }
  // run every module twice on 6 threads concurrently (lazy statics, caches and tables included)
  std::vector<std::thread> ts;
  for (int t = 0; t < 6; ++t)
    ts.emplace_back([t] {
      for (int r = 0; r < 2; ++r) {
        test_hash();
        test_curve();
        if (t < 2) test_pairing();
        test_vrf();
        test_shares_and_ledger();
        test_protocol();
        test_pool(t);
      }
    });
  for (auto& t : ts) t.join();
  std::printf("selftest: %s (%d failures)\n", failures ? "FAILED" : "ok", failures.load());
  return failures ? 1 : 0;
}
