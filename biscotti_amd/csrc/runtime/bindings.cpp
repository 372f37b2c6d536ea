// pybind11 module `_biscotti_rt`: the native host runtime of biscotti_amd.
#include <cstring>
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <cstdlib>
#include <future>
#include <random>
#include <thread>
#include <unordered_map>

#include "bn256.hpp"
#include "hash.hpp"
#include "keys.hpp"
#include "ledger.hpp"
#include "pairing.hpp"
#include "protocol.hpp"
#include "shares.hpp"
#include "vrf.hpp"
#include "pool.hpp"

namespace py = pybind11;
using namespace bsc;

static Bytes B(const py::bytes& b) {
  std::string s = b;
  return Bytes(s.begin(), s.end());
}
static py::bytes P(const Bytes& b) { return py::bytes(reinterpret_cast<const char*>(b.data()), b.size()); }

static U256 u256_from_pyint(const py::int_& v) {
  // accepts non-negative python ints < 2^256
  py::object to_bytes = v.attr("to_bytes");
  py::bytes b = to_bytes(32, "big");
  std::string s = b;
  return U256::from_be(reinterpret_cast<const u8*>(s.data()));
}
static py::int_ pyint_from_u256(const U256& v) {
  Bytes b(32);
  v.to_be(b.data());
  return py::int_(py::module_::import("builtins").attr("int").attr("from_bytes")(P(b), "big"));
}

struct VrfJob {
  std::vector<Bytes> seeds;
  Bytes alpha;
  std::vector<std::pair<Bytes, Bytes>> out;
  std::vector<VrfStage> stages;
  std::string error, beta_error;  // beta_error: set before beta_ready (read by betas())
  std::atomic<bool> finished{false};
  std::promise<void> beta_p;  // every output known (the proofs may still be in progress)
  std::shared_future<void> beta_ready = beta_p.get_future().share();
  std::promise<void> done_p;
  std::shared_future<void> done = done_p.get_future().share();
  std::shared_ptr<VrfJob> after;  // run only once this job has finished (keeps the pool to one job)
  bool outputs_only = false;      // betas only: the proofs are left empty (computed on the device)
  bool started = false;           // handed to the dispatcher: the destructor waits for it
  std::atomic<bool> exited{false};
  std::chrono::steady_clock::time_point t_submit, t_start, t_end;
  ~VrfJob() {
    if (started) {  // the task's last act is setting `exited` (nothing touches the job after it)
      done.wait();
      while (!exited.load(std::memory_order_acquire)) std::this_thread::yield();
    }
  }
};

static void marshal_jac_rows(const uint32_t* jac, const int64_t* idx, size_t n, uint8_t* out);

struct SignJob {
  std::vector<Bytes> msgs, bases, out;
  std::vector<uint32_t> jac;   // messages still as device-layout Jacobian rows: marshalled on the job's thread
  std::vector<Scalar> keys;
  std::vector<int> key_of, ids;
  int threads = 1;
  std::string error;
  std::promise<void> done_p;
  std::shared_future<void> done = done_p.get_future().share();
  bool started = false;
  std::atomic<bool> exited{false};
  std::shared_ptr<VrfJob> after_vrf;  // start only once this VRF batch's outputs are known
  ~SignJob() {
    if (started) {  // the task's last act is setting `exited` (nothing touches the job after it)
      done.wait();
      while (!exited.load(std::memory_order_acquire)) std::this_thread::yield();
    }
  }
};

static std::shared_ptr<SignJob> make_sign_job(std::vector<py::bytes>& msgs, std::vector<py::bytes>& sks,
                                              std::vector<int>& key_of, std::vector<py::bytes>& nonce_base,
                                              std::vector<int>& nonce_ids, int threads) {
  const size_t n = msgs.size();
  if (key_of.size() != n || nonce_ids.size() != n || nonce_base.size() != sks.size())
    throw std::runtime_error("schnorr_sign_multi: length mismatch");
  auto job = std::make_shared<SignJob>();
  for (auto& x : msgs) job->msgs.push_back(B(x));
  for (auto& x : sks) job->keys.push_back(Scalar::from_be(B(x)));
  for (auto& x : nonce_base) job->bases.push_back(B(x));
  for (int k : key_of)
    if (k < 0 || size_t(k) >= job->keys.size()) throw std::runtime_error("schnorr_sign_multi: bad key index");
  job->key_of = key_of;
  job->ids = nonce_ids;
  job->threads = threads;
  job->out.resize(n);
  (void)gen_table();
  return job;
}

static void run_sign_job(SignJob& j);

// messages as rows of one uint8 table (the round's commitments, [n, width]): no bytes object per message
static std::shared_ptr<SignJob> make_sign_job_rows(py::array_t<uint8_t, py::array::c_style | py::array::forcecast> table,
                                                   std::vector<int>& rows, std::vector<py::bytes>& sks,
                                                   std::vector<int>& key_of, std::vector<py::bytes>& nonce_base,
                                                   std::vector<int>& nonce_ids, int threads) {
  if (table.ndim() != 2) throw std::runtime_error("schnorr_sign_rows: table must be [n, width]");
  const size_t nt = size_t(table.shape(0)), wd = size_t(table.shape(1));
  const size_t n = rows.size();
  if (key_of.size() != n || nonce_ids.size() != n || nonce_base.size() != sks.size())
    throw std::runtime_error("schnorr_sign_rows: length mismatch");
  auto job = std::make_shared<SignJob>();
  const uint8_t* t = table.data();
  job->msgs.reserve(n);
  for (int r : rows) {
    if (r < 0 || size_t(r) >= nt) throw std::runtime_error("schnorr_sign_rows: bad row");
    job->msgs.emplace_back(t + size_t(r) * wd, t + (size_t(r) + 1) * wd);
  }
  for (auto& x : sks) job->keys.push_back(Scalar::from_be(B(x)));
  for (auto& x : nonce_base) job->bases.push_back(B(x));
  for (int k : key_of)
    if (k < 0 || size_t(k) >= job->keys.size()) throw std::runtime_error("schnorr_sign_rows: bad key index");
  job->key_of = key_of;
  job->ids = nonce_ids;
  job->threads = threads;
  job->out.resize(n);
  (void)gen_table();
  return job;
}

static void start_sign_job(SignJob* jp) {
  jp->started = true;
  dispatcher().submit([jp] {
    try {
      if (jp->after_vrf) jp->after_vrf->beta_ready.wait();
      jp->after_vrf.reset();
      run_sign_job(*jp);
    } catch (const std::exception& e) {
      jp->error = e.what();
    }
    jp->done_p.set_value();
    jp->exited.store(true, std::memory_order_release);
  });
}

static void run_sign_job(SignJob& j) {
  if (!j.jac.empty()) {   // the messages: commitments marshalled here, off the round's thread
    const size_t nj = j.jac.size() / 24;
    std::vector<uint8_t> m(nj * 64);
    marshal_jac_rows(j.jac.data(), nullptr, nj, m.data());
    j.msgs.resize(nj);
    for (size_t k = 0; k < nj; ++k) j.msgs[k].assign(m.begin() + 64 * k, m.begin() + 64 * (k + 1));
  }
  // nonce points in parallel, ONE inversion for all their marshals, responses in parallel
  const size_t n = j.msgs.size();
  std::vector<Scalar> vs(n);
  std::vector<G1> ts(n);
  parallel_for(n, j.threads, [&](size_t i) {
    Bytes ent = j.bases[size_t(j.key_of[i])];
    const uint32_t id = uint32_t(j.ids[i]);
    for (int b = 0; b < 4; ++b) ent.push_back(u8(id >> (8 * b)));
    auto vt = schnorr_nonce(ent);
    vs[i] = vt.first;
    ts[i] = vt.second;
  });
  const std::vector<Bytes> tm = g1_marshal_batch(ts);
  parallel_for(n, j.threads, [&](size_t i) {
    j.out[i] = schnorr_finish(j.msgs[i], j.keys[size_t(j.key_of[i])], vs[i], tm[i]);
  });
}

// ---------------------------------------------------------------- KZG audit helpers
// r = splitmix64(seed + (idx + 1) * golden) | 1 -- the device kernel derives the same values
static inline u64 kzg_r(u64 seed, u64 idx) {
  u64 z = seed + (idx + 1) * 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return (z ^ (z >> 31)) | 1ull;
}
// signed 192-bit accumulator of r * y products (|sum| < 2^64 * 2^63 * npts)
struct I192 {
  u64 w[3] = {0, 0, 0};
  void add_mul(u64 r, i64 y) {
    const bool neg = y < 0;
    const u64 m = neg ? u64(0) - u64(y) : u64(y);
    const unsigned __int128 p = (unsigned __int128)r * m;
    u64 t[3] = {u64(p), u64(p >> 64), 0};
    if (neg) {  // two's complement of the 192-bit product
      t[0] = ~t[0]; t[1] = ~t[1]; t[2] = ~t[2];
      unsigned __int128 c = (unsigned __int128)t[0] + 1;
      t[0] = u64(c);
      c = (unsigned __int128)t[1] + u64(c >> 64);
      t[1] = u64(c);
      t[2] += u64(c >> 64);
    }
    unsigned __int128 c = (unsigned __int128)w[0] + t[0];
    w[0] = u64(c);
    c = (unsigned __int128)w[1] + t[1] + u64(c >> 64);
    w[1] = u64(c);
    w[2] = w[2] + t[2] + u64(c >> 64);
  }
  bool magnitude(U256& out) const {  // returns true if negative
    const bool neg = w[2] >> 63;
    u64 t[3] = {w[0], w[1], w[2]};
    if (neg) {
      t[0] = ~t[0]; t[1] = ~t[1]; t[2] = ~t[2];
      unsigned __int128 c = (unsigned __int128)t[0] + 1;
      t[0] = u64(c);
      c = (unsigned __int128)t[1] + u64(c >> 64);
      t[1] = u64(c);
      t[2] += u64(c >> 64);
    }
    out = U256();
    out.w[0] = t[0]; out.w[1] = t[1]; out.w[2] = t[2];
    return neg;
  }
};
static std::shared_ptr<G2Prepared> prepared_g2(const Bytes& marshal) {
  static std::mutex mu;
  static std::unordered_map<std::string, std::shared_ptr<G2Prepared>> cache;
  const std::string key(marshal.begin(), marshal.end());
  {
    std::lock_guard<std::mutex> lk(mu);
    auto it = cache.find(key);
    if (it != cache.end()) return it->second;
  }
  auto pr = std::make_shared<G2Prepared>(g2_prepare(G2::unmarshal(marshal)));
  std::lock_guard<std::mutex> lk(mu);
  return cache.emplace(key, pr).first->second;
}
// device Jacobian (8 LE 32-bit limbs per coordinate, Montgomery) -> host G1 (same representation)
static G1 g1_from_dev_jac(const uint32_t* v) {
  G1 g;
  U256* c[3] = {&g.x, &g.y, &g.z};
  for (int i = 0; i < 3; ++i)
    for (int k = 0; k < 4; ++k) c[i]->w[k] = u64(v[8 * i + 2 * k]) | (u64(v[8 * i + 2 * k + 1]) << 32);
  if (g.z.is_zero()) return G1::infinity();
  if (!g.on_curve()) fail("device point is not on the curve");
  return g;
}
struct KzgJob {
  G1 pts[3];
  std::shared_ptr<G2Prepared> q0, q1, qg;
  bool ok = false;
  std::string error;
  std::promise<void> done_p;
  std::shared_future<void> done = done_p.get_future().share();
  bool started = false;
  std::atomic<bool> exited{false};
  ~KzgJob() {
    if (started) {  // the task's last act is setting `exited` (nothing touches the job after it)
      done.wait();
      while (!exited.load(std::memory_order_acquire)) std::this_thread::yield();
    }
  }
};

struct CommitKey {
  std::vector<G1> pk;
  size_t dim() const { return pk.size(); }
};

static py::array_t<uint32_t> g1_affine_u32(const std::vector<G1>& pts) {
  // [n, 16] uint32 : Montgomery affine x (8 LE limbs), y (8 LE limbs); infinity -> zeros
  py::array_t<uint32_t> out({py::ssize_t(pts.size()), py::ssize_t(16)});
  auto o = out.mutable_unchecked<2>();
  for (size_t i = 0; i < pts.size(); ++i) {
    U256 ax, ay;
    pts[i].to_affine(ax, ay);
    for (int k = 0; k < 4; ++k) {
      o(i, 2 * k) = uint32_t(ax.w[k]);
      o(i, 2 * k + 1) = uint32_t(ax.w[k] >> 32);
      o(i, 8 + 2 * k) = uint32_t(ay.w[k]);
      o(i, 8 + 2 * k + 1) = uint32_t(ay.w[k] >> 32);
    }
  }
  return out;
}

static G1 g1_from_jac_u32(const uint32_t* p) {
  G1 g;
  for (int k = 0; k < 4; ++k) {
    g.x.w[k] = u64(p[2 * k]) | (u64(p[2 * k + 1]) << 32);
    g.y.w[k] = u64(p[8 + 2 * k]) | (u64(p[8 + 2 * k + 1]) << 32);
    g.z.w[k] = u64(p[16 + 2 * k]) | (u64(p[16 + 2 * k + 1]) << 32);
  }
  return g;
}

// the IFMA batch path unless BISCOTTI_VRF_SCALAR is set (same-box A/Bs) or the CPU lacks it
static bool vrf_batch_enabled() {
  static const bool on = vrf_beta_batch_supported() && std::getenv("BISCOTTI_VRF_SCALAR") == nullptr;
  return on;
}

// One VRF batch on the native dispatcher: pass 1 computes every output (H, Gamma = x*H, beta), pass 2
// the proofs unless outputs_only (the device prover makes them, kernels/vrf.hip).
static std::shared_ptr<VrfJob> vrf_submit(const std::vector<Bytes>& seeds, const Bytes& alpha, int threads,
                                          std::shared_ptr<VrfJob> after, bool outputs_only,
                                          bool whole_batches = false) {
  auto job = std::make_shared<VrfJob>();
  job->outputs_only = outputs_only;
  job->after = std::move(after);
  job->seeds = seeds;
  job->alpha = alpha;
  job->out.resize(job->seeds.size());
  job->stages.resize(job->seeds.size());
  VrfJob* jp = job.get();
  job->t_submit = std::chrono::steady_clock::now();
  job->started = true;
  dispatcher().submit([jp, threads, whole_batches] {
    if (jp->after) jp->after->done.wait();
    jp->t_start = std::chrono::steady_clock::now();
    bool beta_set = false;
    try {
      // pass 1: every output (H, Gamma = x*H, beta); pass 2: the proofs (k*B, k*H, c, s) unless
      // they are produced elsewhere (outputs_only: the device prover, kernels/vrf.hip)
      const size_t n = jp->seeds.size();
      if (whole_batches && !jp->outputs_only && vrf_batch_enabled()) {
        // outputs AND proofs eight keys at a time (vrf_ifma.cpp prove8): for proofs nothing waits on between
        // the two halves (the run's last round, whose device proofs would outlast it)
        parallel_for((n + 7) / 8, threads, [&](size_t b) {
          const size_t o = 8 * b, m = std::min<size_t>(8, n - o);
          const VrfKey* ks[8];
          Bytes be[8], pi[8];
          for (size_t i = 0; i < m; ++i) ks[i] = &VrfKey::cached(jp->seeds[o + i]);
          vrf_prove_batch(ks, int(m), jp->alpha, be, pi);
          for (size_t i = 0; i < m; ++i) jp->out[o + i] = {std::move(be[i]), std::move(pi[i])};
        });
      } else if (jp->outputs_only && vrf_batch_enabled() && n >= 2 * size_t(std::max(1, threads))) {
        // eight outputs per AVX-512 IFMA batch (vrf_ifma.cpp, ~5x the outputs per core) once each thread would
        // otherwise compute two or more one by one: ~100 outputs on 14 threads take one batch's time
        parallel_for((n + 7) / 8, threads, [&](size_t b) {
          const size_t o = 8 * b, m = std::min<size_t>(8, n - o);
          const VrfKey* ks[8];
          Bytes outs[8];
          for (size_t i = 0; i < m; ++i) ks[i] = &VrfKey::cached(jp->seeds[o + i]);
          vrf_beta_batch(ks, int(m), jp->alpha, outs);
          for (size_t i = 0; i < m; ++i) jp->out[o + i].first = std::move(outs[i]);
        });
      } else if (jp->outputs_only) {
        parallel_for(n, threads, [&](size_t i) {
          jp->out[i].first = vrf_beta(VrfKey::cached(jp->seeds[i]), jp->alpha);
        });
      } else {
        parallel_for(jp->seeds.size(), threads, [&](size_t i) {
          jp->out[i].first = vrf_output(VrfKey::cached(jp->seeds[i]), jp->alpha, &jp->stages[i]);
        });
      }
      jp->beta_p.set_value();
      beta_set = true;
      if (!jp->outputs_only && !(whole_batches && vrf_batch_enabled())) parallel_for(jp->seeds.size(), threads, [&](size_t i) {
        jp->out[i].second = vrf_finish(VrfKey::cached(jp->seeds[i]), jp->stages[i]);
        jp->stages[i].st.reset();
      });
    } catch (const std::exception& e) {
      jp->error = e.what();
      if (!beta_set) jp->beta_error = jp->error;
    }
    if (!beta_set) jp->beta_p.set_value();
    jp->t_end = std::chrono::steady_clock::now();
    jp->finished.store(true);
    jp->after.reset();
    jp->done_p.set_value();
    jp->exited.store(true, std::memory_order_release);
  });
  return job;
}

// a fixed list of VRF seeds held natively (a rank's peers): a batch over it copies no Python objects
// (a 100-seed list cost ~20 us of conversion per submission on the round's host thread)
struct VrfSeedSet {
  std::vector<Bytes> seeds;
};

// the noiser lottery over a VRF batch's outputs (select_noisers_job / RoundFSM.select_noisers_job)
static py::array_t<int64_t> select_noisers_impl(const std::map<i64, i64>& stake, VrfJob& job,
                                                std::vector<i64> out_index, std::vector<i64> selfs, i64 nn,
                                                i64 n) {
  if (job.beta_ready.wait_for(std::chrono::seconds(0)) != std::future_status::ready) {
    py::gil_scoped_release rel;
    job.beta_ready.wait();
  }
  if (!job.beta_error.empty()) throw std::runtime_error(job.beta_error);
  const size_t k = selfs.size();
  if (!out_index.empty() && out_index.size() != k) throw std::runtime_error("select_noisers_job: index length");
  const Lottery table(stake, n, Bytes{});
  const i64 holders = i64(table.ids.size());
  py::array_t<int64_t> res({py::ssize_t(k), py::ssize_t(nn)});
  int64_t* o = res.mutable_data();
  Bytes input;
  input.reserve(64);
  for (size_t w = 0; w < k; ++w) {
    const size_t src = out_index.empty() ? w : size_t(out_index[w]);
    if (src >= job.out.size()) throw std::runtime_error("select_noisers_job: output index out of range");
    const Bytes& beta = job.out[src].first;
    const i64 self = selfs[w];
    const i64 others = holders - (std::binary_search(table.ids.begin(), table.ids.end(), self) ? 1 : 0);
    if (others < nn) throw std::runtime_error("lottery: not enough peers for noisers");
    input.assign(beta.begin(), beta.end());
    size_t i = 0;
    i64 got = 0;
    while (got < nn) {   // Lottery::draw over the shared ticket table
      if (i + 1 >= input.size()) {
        input = Sha256::digest(input);
        i = 0;
      }
      const i64 idx = i64((size_t(input[i]) * 256 + size_t(input[i + 1])) % size_t(table.total()));
      ++i;
      const i64 c = table.ticket(idx);
      bool dup = c == self;
      for (i64 q = 0; q < got && !dup; ++q) dup = o[w * nn + q] == c;
      if (!dup) o[w * nn + got++] = c;
    }
  }
  return res;
}

// Jacobian rows (device layout: [*, 24] Montgomery u32 limbs; rows idx[0..n) of `jac`, or the first n when idx
// is null) -> 64-byte kyber marshals in `out` [n, 64], with ONE inversion (Montgomery's trick)
static void marshal_jac_rows(const uint32_t* jac, const int64_t* idx, size_t n, uint8_t* out) {
  std::vector<G1> pts(n);
  for (size_t i = 0; i < n; ++i) pts[i] = g1_from_jac_u32(jac + 24 * size_t(idx != nullptr ? idx[i] : int64_t(i)));
  const MontField& F = Fp();
  std::vector<U256> pre(n);
  U256 acc = F.one;
  for (size_t i = 0; i < n; ++i) {
    pre[i] = acc;
    if (!pts[i].is_inf()) F.mul(acc, acc, pts[i].z);
  }
  U256 inv;
  F.inv_mont(inv, acc);
  std::memset(out, 0, n * 64);
  for (size_t k = n; k-- > 0;) {
    if (pts[k].is_inf()) continue;
    U256 zi, zi2, zi3, ax, ay;
    F.mul(zi, inv, pre[k]);
    F.mul(inv, inv, pts[k].z);
    F.sqr(zi2, zi);
    F.mul(zi3, zi2, zi);
    F.mul(ax, pts[k].x, zi2);
    F.mul(ay, pts[k].y, zi3);
    F.from_mont(ax).to_be(out + 64 * k);
    F.from_mont(ay).to_be(out + 64 * k + 32);
  }
}

PYBIND11_MODULE(_biscotti_rt, m) {
  m.doc() = "biscotti_amd native host runtime (crypto, ledger, protocol FSM)";

  // ---------------------------------------------------------------- hashing
  m.def("sha256", [](py::bytes d) { return P(Sha256::digest(B(d))); });
  m.def("sha512", [](py::bytes d) { return P(Sha512::digest(B(d))); });
  m.def("blake2b", [](py::bytes d, int outlen, py::bytes key) {
    Bytes k = B(key), x = B(d);
    Blake2b h;
    h.init(size_t(outlen), k.data(), k.size());
    h.update(x.data(), x.size());
    Bytes o(static_cast<size_t>(outlen));
    h.final(o.data());
    return P(o);
  }, py::arg("data"), py::arg("outlen") = 64, py::arg("key") = py::bytes(""));
  m.def("blake2b_param", [](py::bytes param, py::bytes d) {
    Bytes p = B(param), x = B(d);
    if (p.size() != 64) throw std::runtime_error("param block must be 64 bytes");
    Blake2b h;
    h.init_param(p.data(), nullptr, 0);
    h.update(x.data(), x.size());
    Bytes o(h.outlen);
    h.final(o.data());
    return P(o);
  });
  m.def("blake2xb", [](py::bytes seed, py::bytes msg, size_t n) {
    Blake2Xb x(B(seed));
    x.write(B(msg));
    Bytes o(n);
    x.read(o.data(), n);
    return P(o);
  });

  // ---------------------------------------------------------------- bn256
  m.def("bn256_prime", [] { return pyint_from_u256(PRIME()); });
  m.def("bn256_order", [] { return pyint_from_u256(ORDER()); });
  m.def("g1_generator", [] { return P(G1::generator().marshal()); });
  m.def("g1_infinity", [] { return P(G1::infinity().marshal()); });
  m.def("g1_add", [](py::bytes a, py::bytes b) { return P(G1::unmarshal(B(a)).add(G1::unmarshal(B(b))).marshal()); });
  m.def("g1_neg", [](py::bytes a) { return P(G1::unmarshal(B(a)).neg().marshal()); });
  m.def("g1_mul", [](py::bytes a, py::int_ k) { return P(G1::unmarshal(B(a)).mul(u256_from_pyint(k)).marshal()); });
  m.def("g1_mul_i64", [](py::bytes a, int64_t k) { return P(G1::unmarshal(B(a)).mul_i64(k).marshal()); });
  m.def("g1_base_mul", [](py::int_ k) { return P(gen_table().mul(u256_from_pyint(k)).marshal()); });
  m.def("g1_is_valid", [](py::bytes a) {
    try { G1::unmarshal(B(a)); return true; } catch (...) { return false; }
  });
  m.def("g1_affine_mont_u32", [](py::bytes a) { return g1_affine_u32({G1::unmarshal(B(a))}); });
  m.def("g1_marshal_jac_u32", [](py::array_t<uint32_t, py::array::c_style | py::array::forcecast> jac) {
    // [n, 24] Montgomery Jacobian limbs (device layout) -> list of 64-byte marshals
    if (jac.ndim() != 2 || jac.shape(1) != 24) throw std::runtime_error("expected [n, 24] uint32");
    py::list out;
    for (py::ssize_t i = 0; i < jac.shape(0); ++i) out.append(P(g1_from_jac_u32(jac.data(i, 0)).marshal()));
    return out;
  });
  m.def("g1_marshal_jac_batch", [](py::array_t<uint32_t, py::array::c_style | py::array::forcecast> jac) {
    // [n, 24] device Jacobian limbs -> uint8 [n, 64] marshals with ONE inversion (Montgomery's trick)
    if (jac.ndim() != 2 || jac.shape(1) != 24) throw std::runtime_error("expected [n, 24] uint32");
    const size_t n = size_t(jac.shape(0));
    py::array_t<uint8_t> out({py::ssize_t(n), py::ssize_t(64)});
    marshal_jac_rows(jac.data(), nullptr, n, out.mutable_data());
    return out;
  });
  m.def("g1_sum_jac_u32", [](py::array_t<uint32_t, py::array::c_style | py::array::forcecast> jac) {
    G1 acc = G1::infinity();
    for (py::ssize_t i = 0; i < jac.shape(0); ++i) acc = acc.add(g1_from_jac_u32(jac.data(i, 0)));
    return P(acc.marshal());
  });
  m.def("g1_sum_marshaled", [](py::array_t<uint8_t, py::array::c_style | py::array::forcecast> a) {
    // a: [R, C, 64] marshaled points -> [C, 64] sums over R (miner-side aggregateSecret on CPU)
    if (a.ndim() != 3 || a.shape(2) != 64) throw std::runtime_error("expected [R, C, 64] uint8");
    const py::ssize_t R = a.shape(0), Cn = a.shape(1);
    py::array_t<uint8_t> out({Cn, py::ssize_t(64)});
    std::vector<G1> acc(size_t(Cn), G1::infinity());
    {
      py::gil_scoped_release rel;
      for (py::ssize_t c = 0; c < Cn; ++c)
        for (py::ssize_t r = 0; r < R; ++r)
          acc[size_t(c)] = acc[size_t(c)].add(G1::unmarshal(Bytes(a.data(r, c, 0), a.data(r, c, 0) + 64)));
    }
    for (py::ssize_t c = 0; c < Cn; ++c) {
      Bytes b = acc[size_t(c)].marshal();
      std::memcpy(out.mutable_data(c, 0), b.data(), 64);
    }
    return out;
  });
  m.def("g2_generator", [] { return P(G2::generator().marshal()); });
  m.def("g2_mul", [](py::bytes a, py::int_ k) { return P(G2::unmarshal(B(a)).mul(u256_from_pyint(k)).marshal()); });
  m.def("g2_add", [](py::bytes a, py::bytes b) { return P(G2::unmarshal(B(a)).add(G2::unmarshal(B(b))).marshal()); });
  m.def("g2_is_valid", [](py::bytes a) {
    try { G2::unmarshal(B(a)); return true; } catch (...) { return false; }
  });
  m.def("scalar_from_i64", [](int64_t v) { return P(Scalar::from_i64(v).to_be()); });

  // ---------------------------------------------------------------- Schnorr
  m.def("schnorr_sign", [](py::bytes msg, py::bytes sk, py::bytes nonce) {
    return P(schnorr_sign(B(msg), Scalar::from_be(B(sk)), B(nonce)));
  });
  m.def("schnorr_verify", [](py::bytes msg, py::bytes pk, py::bytes sig) {
    return schnorr_verify(B(msg), G1::unmarshal(B(pk)), B(sig));
  });
  m.def("schnorr_sign_batch", [](std::vector<py::bytes> msgs, py::bytes sk, std::vector<py::bytes> nonces, int threads) {
    std::vector<Bytes> ms, ns, out(msgs.size());
    for (auto& x : msgs) ms.push_back(B(x));
    for (auto& x : nonces) ns.push_back(B(x));
    Scalar s = Scalar::from_be(B(sk));
    (void)gen_table();
    {
      py::gil_scoped_release rel;
      // nonce points in parallel, ONE inversion for all their marshals, responses in parallel
      if (ms.size() != ns.size()) throw std::runtime_error("messages / nonces length mismatch");
      std::vector<Scalar> vs(ms.size());
      std::vector<G1> ts(ms.size());
      parallel_for(ms.size(), threads, [&](size_t i) {
        auto vt = schnorr_nonce(ns[i]);
        vs[i] = vt.first;
        ts[i] = vt.second;
      });
      const std::vector<Bytes> tm = g1_marshal_batch(ts);
      parallel_for(ms.size(), threads, [&](size_t i) { out[i] = schnorr_finish(ms[i], s, vs[i], tm[i]); });
    }
    std::vector<py::bytes> r;
    for (auto& o : out) r.push_back(P(o));
    return r;
  });
  // All signatures of a round in one call: message i signed with sks[key_of[i]], nonce entropy
  // nonce_base[key_of[i]] || le32(nonce_ids[i]).  _async returns a job that signs on native
  // threads right away (result() joins) so the work overlaps the GPU share computation.
  py::class_<SignJob, std::shared_ptr<SignJob>>(m, "SignJob")
      .def("result", [](SignJob& j) {
        {
          py::gil_scoped_release rel;
          j.done.wait();
        }
        if (!j.error.empty()) throw std::runtime_error(j.error);
        std::vector<py::bytes> r;
        for (auto& o : j.out) r.push_back(P(o));
        return r;
      })
      // every signature as one uint8 [n, 64] array (one allocation instead of n bytes objects)
      .def("result_array", [](SignJob& j) {
        {
          py::gil_scoped_release rel;
          j.done.wait();
        }
        if (!j.error.empty()) throw std::runtime_error(j.error);
        py::array_t<uint8_t> a({py::ssize_t(j.out.size()), py::ssize_t(64)});
        uint8_t* o = a.mutable_data();
        for (size_t i = 0; i < j.out.size(); ++i) {
          if (j.out[i].size() != 64) throw std::runtime_error("signature is not 64 bytes");
          std::memcpy(o + 64 * i, j.out[i].data(), 64);
        }
        return a;
      });
  m.def("schnorr_sign_multi", [](std::vector<py::bytes> msgs, std::vector<py::bytes> sks, std::vector<int> key_of,
                                 std::vector<py::bytes> nonce_base, std::vector<int> nonce_ids, int threads) {
    auto job = make_sign_job(msgs, sks, key_of, nonce_base, nonce_ids, threads);
    {
      py::gil_scoped_release rel;
      run_sign_job(*job);
    }
    std::vector<py::bytes> r;
    for (auto& o : job->out) r.push_back(P(o));
    return r;
  });
  m.def("schnorr_sign_multi_async", [](std::vector<py::bytes> msgs, std::vector<py::bytes> sks,
                                       std::vector<int> key_of, std::vector<py::bytes> nonce_base,
                                       std::vector<int> nonce_ids, int threads) {
    auto job = make_sign_job(msgs, sks, key_of, nonce_base, nonce_ids, threads);
    start_sign_job(job.get());
    return job;
  });
  // same, message i = table[rows[i]] (e.g. the marshalled commitments of the round, uint8 [n, 64])
  m.def("schnorr_sign_rows_async", [](py::array_t<uint8_t, py::array::c_style | py::array::forcecast> table,
                                      std::vector<int> rows, std::vector<py::bytes> sks, std::vector<int> key_of,
                                      std::vector<py::bytes> nonce_base, std::vector<int> nonce_ids, int threads,
                                      std::shared_ptr<VrfJob> after_vrf) {
    // after_vrf: the signatures yield the host threads to a VRF batch whose outputs gate the next
    // round (they start once its outputs are known)
    auto job = make_sign_job_rows(table, rows, sks, key_of, nonce_base, nonce_ids, threads);
    job->after_vrf = std::move(after_vrf);
    start_sign_job(job.get());
    return job;
  }, py::arg("table"), py::arg("rows"), py::arg("sks"), py::arg("key_of"), py::arg("nonce_base"),
     py::arg("nonce_ids"), py::arg("threads"), py::arg("after_vrf") = nullptr);
  // the same with the table as device-layout Jacobian rows [n, 24] uint32 (the pre-step's read-back): the
  // signed rows are copied now and marshalled on the job's thread
  m.def("schnorr_sign_rows_jac_async", [](py::array_t<uint32_t, py::array::c_style | py::array::forcecast> jac,
                                          std::vector<int> rows, std::vector<py::bytes> sks, std::vector<int> key_of,
                                          std::vector<py::bytes> nonce_base, std::vector<int> nonce_ids, int threads,
                                          std::shared_ptr<VrfJob> after_vrf) {
    if (jac.ndim() != 2 || jac.shape(1) != 24) throw std::runtime_error("schnorr_sign_rows_jac: expected [n, 24]");
    const size_t n = rows.size();
    if (key_of.size() != n || nonce_ids.size() != n || nonce_base.size() != sks.size())
      throw std::runtime_error("schnorr_sign_rows_jac: length mismatch");
    auto job = std::make_shared<SignJob>();
    job->jac.resize(n * 24);
    for (size_t i = 0; i < n; ++i) {
      if (rows[i] < 0 || rows[i] >= jac.shape(0)) throw std::runtime_error("schnorr_sign_rows_jac: bad row");
      std::memcpy(job->jac.data() + 24 * i, jac.data(rows[i], 0), 24 * sizeof(uint32_t));
    }
    for (auto& x : sks) job->keys.push_back(Scalar::from_be(B(x)));
    for (auto& x : nonce_base) job->bases.push_back(B(x));
    for (int k : key_of)
      if (k < 0 || size_t(k) >= job->keys.size()) throw std::runtime_error("schnorr_sign_rows_jac: bad key index");
    job->key_of = key_of;
    job->ids = nonce_ids;
    job->threads = threads;
    job->out.resize(n);
    (void)gen_table();
    job->after_vrf = std::move(after_vrf);
    start_sign_job(job.get());
    return job;
  }, py::arg("jac"), py::arg("rows"), py::arg("sks"), py::arg("key_of"), py::arg("nonce_base"),
     py::arg("nonce_ids"), py::arg("threads"), py::arg("after_vrf") = nullptr);
  m.def("client_key_from_entropy", [](py::bytes e) {
    auto kp = client_key_from_entropy(B(e));
    return py::make_tuple(P(kp.first.to_be()), P(kp.second.marshal()));
  });

  // ---------------------------------------------------------------- pairing (kyber.go:650-673)
  auto gt_bytes = [](const Fp12& g) {
    Bytes out;
    for (int k = 0; k < 6; ++k)
      for (const U256* v : {&g.c[k].x, &g.c[k].y}) {
        u8 b[32];
        Fp().from_mont(*v).to_be(b);
        out.insert(out.end(), b, b + 32);
      }
    return out;
  };
  m.def("pairing_digest", [gt_bytes](py::bytes g1, py::bytes g2, py::int_ k) {
    // e(P, Q)^k as 384 canonical bytes (GT equality tests; kyber's GT marshal is not reproduced)
    Fp12 g;
    {
      G1 P = G1::unmarshal(B(g1));
      G2 Q = G2::unmarshal(B(g2));
      U256 e = u256_from_pyint(k);
      py::gil_scoped_release rel;
      g = pairing(P, Q).pow(e);
    }
    return P(gt_bytes(g));
  }, py::arg("g1"), py::arg("g2"), py::arg("k") = 1);
  m.def("pairing_product_is_one", [](std::vector<py::bytes> g1s, std::vector<py::bytes> g2s) {
    std::vector<G1> Ps;
    std::vector<G2> Qs;
    for (auto& b : g1s) Ps.push_back(G1::unmarshal(B(b)));
    for (auto& b : g2s) Qs.push_back(G2::unmarshal(B(b)));
    py::gil_scoped_release rel;
    return multi_pairing(Ps, Qs).is_one();
  });
  m.def("verify_secret", [](py::bytes commitment, py::bytes witness, py::bytes g2_0, py::bytes g2_1, i64 x, i64 y,
                            py::object y_base) {
    G1 C = G1::unmarshal(B(commitment)), W = G1::unmarshal(B(witness));
    G2 A = G2::unmarshal(B(g2_0)), S = G2::unmarshal(B(g2_1));
    G1 Yb = y_base.is_none() ? G1::generator() : G1::unmarshal(B(y_base.cast<py::bytes>()));
    py::gil_scoped_release rel;
    return verify_secret(C, W, A, S, x, y, Yb);
  }, py::arg("commitment"), py::arg("witness"), py::arg("g2_0"), py::arg("g2_1"), py::arg("x"), py::arg("y"),
     py::arg("y_base") = py::none());
  m.def("verify_secrets_batch", [](std::vector<py::bytes> commits, std::vector<py::bytes> witnesses, py::bytes g2_0,
                                   py::bytes g2_1, std::vector<i64> xs, std::vector<i64> ys, int threads,
                                   py::object y_base) {
    const size_t n = commits.size();
    if (witnesses.size() != n || xs.size() != n || ys.size() != n) throw std::runtime_error("length mismatch");
    std::vector<G1> C, W;
    for (auto& b : commits) C.push_back(G1::unmarshal(B(b)));
    for (auto& b : witnesses) W.push_back(G1::unmarshal(B(b)));
    G2 A = G2::unmarshal(B(g2_0)), S = G2::unmarshal(B(g2_1));
    G1 Yb = y_base.is_none() ? G1::generator() : G1::unmarshal(B(y_base.cast<py::bytes>()));
    std::vector<uint8_t> ok(n, 0);
    {
      py::gil_scoped_release rel;
      parallel_for(n, threads, [&](size_t i) { ok[i] = verify_secret(C[i], W[i], A, S, xs[i], ys[i], Yb) ? 1 : 0; });
    }
    std::vector<bool> r(ok.begin(), ok.end());
    return r;
  }, py::arg("commits"), py::arg("witnesses"), py::arg("g2_0"), py::arg("g2_1"), py::arg("xs"), py::arg("ys"),
     py::arg("threads") = 1, py::arg("y_base") = py::none());

  // ---------------------------------------------------------------- batched KZG audit (K13)
  // verifySecret (kyber.go:650-673) over every (chunk k, share point j) of an aggregate at once:
  // with random 64-bit r_kj the checks e(C_k - y_kj B_k, g2_0) == e(W_kj, g2_1 - x_j G2) collapse to
  //   e(L1, g2_0) * e(-A, g2_1) * e(L2, G2) == 1,
  //   L1 = sum_k (R_k C_k - Z_k B_k), R_k = sum_j r_kj, Z_k = sum_j r_kj y_kj,
  //   A = sum r_kj W_kj,  L2 = sum x_j r_kj W_kj.
  // The device computes the three points (kernels/kzg.hip); kzg_rlc_host is the CPU path and the
  // test oracle.  r_kj = kzg_r(seed, k * npts + j) on both sides.
  m.def("kzg_r", [](u64 seed, u64 idx) { return kzg_r(seed, idx); });
  m.def("kzg_rlc_host", [](std::vector<py::bytes> commits, std::vector<py::bytes> wits,
                           py::array_t<int64_t, py::array::c_style | py::array::forcecast> ys, std::vector<i64> xs,
                           std::vector<py::bytes> bases, u64 seed, int threads) {
    const size_t nch = commits.size(), npts = xs.size();
    if (wits.size() != nch * npts || size_t(ys.size()) != nch * npts || (bases.size() != 1 && bases.size() != nch))
      throw std::runtime_error("kzg_rlc_host: shape mismatch");
    std::vector<G1> C, W, Bs;
    for (auto& b : commits) C.push_back(G1::unmarshal(B(b)));
    for (auto& b : wits) W.push_back(G1::unmarshal(B(b)));
    for (auto& b : bases) Bs.push_back(G1::unmarshal(B(b)));
    const int64_t* y = ys.data();
    std::vector<G1> l1(nch), a(nch), l2(nch);
    {
      py::gil_scoped_release rel;
      parallel_for(nch, threads, [&](size_t k) {
        G1 acc_a = G1::infinity(), acc_l2 = G1::infinity();
        unsigned __int128 R = 0;
        I192 Z;
        for (size_t j = 0; j < npts; ++j) {
          const u64 r = kzg_r(seed, k * npts + j);
          const G1 rw = W[k * npts + j].mul(U256::from_u64(r));
          acc_a = acc_a.add(rw);
          acc_l2 = acc_l2.add(rw.mul_i64(xs[j]));
          R += r;
          Z.add_mul(r, y[k * npts + j]);
        }
        U256 Ru;
        Ru.w[0] = u64(R);
        Ru.w[1] = u64(R >> 64);
        U256 Zm;
        const bool zneg = Z.magnitude(Zm);
        const G1 zb = Bs[Bs.size() == 1 ? 0 : k].mul(Zm);
        l1[k] = C[k].mul(Ru).add(zneg ? zb : zb.neg());
        a[k] = acc_a;
        l2[k] = acc_l2;
      });
    }
    G1 L1 = G1::infinity(), A = G1::infinity(), L2 = G1::infinity();
    for (size_t k = 0; k < nch; ++k) { L1 = L1.add(l1[k]); A = A.add(a[k]); L2 = L2.add(l2[k]); }
    return py::make_tuple(P(L1.marshal()), P(A.marshal()), P(L2.marshal()));
  }, py::arg("commits"), py::arg("witnesses"), py::arg("ys"), py::arg("xs"), py::arg("bases"), py::arg("seed"),
     py::arg("threads") = 1);
  m.def("kzg_check", [](py::bytes l1, py::bytes a, py::bytes l2, py::bytes g2_0, py::bytes g2_1) {
    G1 L1 = G1::unmarshal(B(l1)), A = G1::unmarshal(B(a)), L2 = G1::unmarshal(B(l2));
    auto q0 = prepared_g2(B(g2_0)), q1 = prepared_g2(B(g2_1)), qg = prepared_g2(G2::generator().marshal());
    py::gil_scoped_release rel;
    return multi_pairing_is_one({L1, A.neg(), L2}, {q0.get(), q1.get(), qg.get()});
  });
  // the device result: int32/uint32 [3, 24] Jacobian Montgomery (L1, A, L2); the pairing product
  // runs on a native thread (result() joins) so it overlaps the next round
  py::class_<KzgJob, std::shared_ptr<KzgJob>>(m, "KzgJob").def("result", [](KzgJob& j) {
    {
      py::gil_scoped_release rel;
      j.done.wait();
    }
    if (!j.error.empty()) throw std::runtime_error(j.error);
    return j.ok;
  });
  m.def("kzg_check_device_async", [](py::array_t<uint32_t, py::array::c_style | py::array::forcecast> pts,
                                     py::bytes g2_0, py::bytes g2_1) {
    if (pts.size() != 72) throw std::runtime_error("kzg_check_device_async: expected [3, 24] limbs");
    auto job = std::make_shared<KzgJob>();
    for (int i = 0; i < 3; ++i) job->pts[i] = g1_from_dev_jac(pts.data() + 24 * i);
    job->q0 = prepared_g2(B(g2_0));
    job->q1 = prepared_g2(B(g2_1));
    job->qg = prepared_g2(G2::generator().marshal());
    KzgJob* jp = job.get();
    jp->started = true;
    dispatcher().submit([jp] {
      try {
        jp->ok = multi_pairing_is_one({jp->pts[0], jp->pts[1].neg(), jp->pts[2]},
                                      {jp->q0.get(), jp->q1.get(), jp->qg.get()});
      } catch (const std::exception& e) {
        jp->error = e.what();
      }
      jp->done_p.set_value();
      jp->exited.store(true, std::memory_order_release);
    });
    return job;
  });
  m.def("g1_from_device_jac", [](py::array_t<uint32_t, py::array::c_style | py::array::forcecast> v) {
    if (v.size() != 24) throw std::runtime_error("g1_from_device_jac: expected 24 limbs");
    return P(g1_from_dev_jac(v.data()).marshal());
  });
  m.def("final_exp_selftest", [](int n, u64 seed) {
    // the u-chain hard part against the generic 760-bit exponent on Miller-loop outputs
    std::mt19937_64 rng(seed);
    for (int i = 0; i < n; ++i) {
      U256 a, b;
      for (int w = 0; w < 4; ++w) { a.w[w] = rng(); b.w[w] = rng(); }
      a.w[3] >>= 3; b.w[3] >>= 3;
      const G1 P1 = G1::generator().mul(a);
      const G2Prepared q = g2_prepare(G2::generator().mul(b));
      const Fp12 f = miller_prepared({P1}, {&q});
      if (!(final_exp_u(f) == final_exp_generic(f))) return false;
    }
    return true;
  });

  // ---------------------------------------------------------------- VRF
  m.def("vrf_public_key", [](py::bytes seed) { return P(VrfKey::from_seed(B(seed)).pk); });
  m.def("ed25519_public_key", [](py::bytes seed) { return P(ed25519_public_from_seed(B(seed))); });
  m.def("vrf_prove", [](py::bytes seed, py::bytes alpha) {
    auto r = vrf_prove(VrfKey::cached(B(seed)), B(alpha));
    return py::make_tuple(P(r.first), P(r.second));
  });
  m.def("vrf_verify", [](py::bytes pk, py::bytes alpha, py::bytes pi) -> py::object {
    Bytes beta;
    if (!vrf_verify(B(pk), B(alpha), B(pi), &beta)) return py::none();
    return P(beta);
  });
  m.def("vrf_prove_batch", [](std::vector<py::bytes> seeds, py::bytes alpha, int threads) {
    std::vector<Bytes> ss;
    for (auto& s : seeds) ss.push_back(B(s));
    Bytes a = B(alpha);
    std::vector<std::pair<Bytes, Bytes>> out(ss.size());
    {
      py::gil_scoped_release rel;
      parallel_for(ss.size(), threads, [&](size_t i) { out[i] = vrf_prove(VrfKey::cached(ss[i]), a); });
    }
    py::list r;
    for (auto& o : out) r.append(py::make_tuple(P(o.first), P(o.second)));
    return r;
  });
  // Asynchronous batch: proving starts on a native thread immediately (no GIL hand-off, so it
  // overlaps with the caller's GPU work from the first microsecond); result() joins.
  py::class_<VrfJob, std::shared_ptr<VrfJob>>(m, "VrfJob")
      .def("done", [](VrfJob& j) { return j.finished.load(); })
      .def("timing_us", [](VrfJob& j) {  // (submit -> start, start -> end), valid after result()
        auto us = [](auto a, auto b) { return std::chrono::duration<double, std::micro>(b - a).count(); };
        return py::make_tuple(us(j.t_submit, j.t_start), us(j.t_start, j.t_end));
      })
      .def("result", [](VrfJob& j) {
        {
          py::gil_scoped_release rel;
          j.done.wait();
        }
        if (!j.error.empty()) throw std::runtime_error(j.error);
        py::list r;
        for (auto& o : j.out) r.append(py::make_tuple(P(o.first), P(o.second)));
        return r;
      })
      // join without materialising the proofs as Python objects (callers that discard them); a finished
      // job is joined without the GIL round trip
      .def("wait", [](VrfJob& j) {
        if (!j.finished.load(std::memory_order_acquire)) {
          py::gil_scoped_release rel;
          j.done.wait();
        }
        if (!j.error.empty()) throw std::runtime_error(j.error);
      })
      // the outputs only: returns as soon as every Gamma = x*H is known, while the proofs finish
      .def("betas", [](VrfJob& j) {
        {
          py::gil_scoped_release rel;
          j.beta_ready.wait();
        }
        if (!j.beta_error.empty()) throw std::runtime_error(j.beta_error);
        py::list r;
        for (auto& o : j.out) r.append(P(o.first));
        return r;
      });
  m.def("vrf_key_material", [](py::bytes seed) {
    // x (clamped secret) || nonce prefix || encoded public key: the device prover's key row
    const VrfKey& k = VrfKey::cached(B(seed));
    Bytes out(k.x, k.x + 32);
    out.insert(out.end(), k.prefix, k.prefix + 32);
    out.insert(out.end(), k.pk.begin(), k.pk.end());
    return P(out);
  });
  m.def("vrf_base_table", [] { return P(vrf_base_table_bytes()); });
  m.def("vrf_beta", [](py::bytes seed, py::bytes alpha) { return P(vrf_beta(VrfKey::cached(B(seed)), B(alpha))); });
  m.def("vrf_beta_batch_supported", [] { return vrf_beta_batch_supported(); });
  m.def("vrf_beta_batch", [](std::vector<py::bytes> seeds, py::bytes alpha) {
    std::vector<const VrfKey*> ks;
    for (auto& s : seeds) ks.push_back(&VrfKey::cached(B(s)));
    const Bytes a = B(alpha);
    std::vector<Bytes> out(ks.size());
    {
      py::gil_scoped_release rel;
      vrf_beta_batch(ks.data(), int(ks.size()), a, out.data());
    }
    py::list res;
    for (auto& o : out) res.append(P(o));
    return res;
  });
  py::class_<VrfSeedSet, std::shared_ptr<VrfSeedSet>>(m, "VrfSeedSet")
      .def(py::init([](std::vector<py::bytes> seeds) {
        auto st = std::make_shared<VrfSeedSet>();
        for (auto& x : seeds) st->seeds.push_back(B(x));
        return st;
      }))
      .def("__len__", [](const VrfSeedSet& st) { return st.seeds.size(); });
  m.def("vrf_prove_set_async", [](std::shared_ptr<VrfSeedSet> set, py::bytes alpha, int threads,
                                  std::shared_ptr<VrfJob> after, bool outputs_only) {
    return vrf_submit(set->seeds, B(alpha), threads, std::move(after), outputs_only);
  }, py::arg("seeds"), py::arg("alpha"), py::arg("threads"), py::arg("after") = nullptr,
     py::arg("outputs_only") = false);
  m.def("vrf_prove_batch_async", [](std::vector<py::bytes> seeds, py::bytes alpha, int threads,
                                    std::shared_ptr<VrfJob> after, bool outputs_only) {
    std::vector<Bytes> ss;
    for (auto& x : seeds) ss.push_back(B(x));
    return vrf_submit(ss, B(alpha), threads, std::move(after), outputs_only);
  }, py::arg("seeds"), py::arg("alpha"), py::arg("threads"), py::arg("after") = nullptr,
     py::arg("outputs_only") = false);
  // outputs + proofs in whole 8-key batches on AVX-512 IFMA (vrf_prove_batch), the outputs known only at the end:
  // for proofs nobody reads before the job's join (the run's last round, engine._round_front)
  m.def("vrf_proofs_async", [](std::vector<py::bytes> seeds, py::bytes alpha, int threads) {
    std::vector<Bytes> ss;
    for (auto& x : seeds) ss.push_back(B(x));
    return vrf_submit(ss, B(alpha), threads, nullptr, false, true);
  }, py::arg("seeds"), py::arg("alpha"), py::arg("threads"));
  m.def("vrf_prove_batch_ifma", [](std::vector<py::bytes> seeds, py::bytes alpha) {
    std::vector<const VrfKey*> ks;
    for (auto& s : seeds) ks.push_back(&VrfKey::cached(B(s)));
    const Bytes a = B(alpha);
    std::vector<Bytes> be(ks.size()), pi(ks.size());
    {
      py::gil_scoped_release rel;
      vrf_prove_batch(ks.data(), int(ks.size()), a, be.data(), pi.data());
    }
    py::list res;
    for (size_t i = 0; i < ks.size(); ++i) res.append(py::make_tuple(P(be[i]), P(pi[i])));
    return res;
  });

  // ---------------------------------------------------------------- keys
  py::class_<CommitKey>(m, "CommitKey")
      .def_static("generate", [](size_t d, int64_t s) {
        CommitKey k; k.pk = gen_commit_key_g1(d, Scalar::from_i64(s)); return k;
      }, py::arg("d"), py::arg("secret") = 2)
      .def_static("load", [](const std::string& path, size_t d, bool check_g2) {
        CommitKey k; k.pk = read_commit_key(path, d, check_g2); return k;
      }, py::arg("path"), py::arg("d"), py::arg("check_g2") = false)
      .def_static("from_points", [](std::vector<py::bytes> pts) {
        CommitKey k; for (auto& p : pts) k.pk.push_back(G1::unmarshal(B(p))); return k;
      })
      .def("__len__", &CommitKey::dim)
      .def("point", [](const CommitKey& k, size_t i) { return P(k.pk.at(i).marshal()); })
      .def("affine_mont_u32", [](const CommitKey& k) { return g1_affine_u32(k.pk); })
      .def("witness_bases_affine_u32", [](const CommitKey& k, int64_t poly, int64_t total) {
        return g1_affine_u32(witness_bases(k.pk, int64_t(k.pk.size()), poly, total));
      })
      .def("commit", [](const CommitKey& k, py::array_t<int64_t, py::array::c_style | py::array::forcecast> c, size_t off) {
        std::vector<i64> v(c.data(), c.data() + c.size());
        G1 r;
        { py::gil_scoped_release rel; r = commit(v, k.pk, off); }
        return P(r.marshal());
      }, py::arg("coeffs"), py::arg("offset") = 0)
      .def("make_shares", [](const CommitKey& k, py::array_t<int64_t, py::array::c_style | py::array::forcecast> c,
                             int64_t poly, int64_t total) {
        std::vector<i64> v(c.data(), c.data() + c.size());
        SharePackage sp;
        { py::gil_scoped_release rel; sp = make_shares(v, k.pk, poly, total); }
        size_t nch = sp.chunk_commit.size();
        py::array_t<int64_t> ys({py::ssize_t(nch), py::ssize_t(total)});
        std::memcpy(ys.mutable_data(), sp.ys.data(), sp.ys.size() * 8);
        py::list cc, wit;
        for (auto& g : sp.chunk_commit) cc.append(P(g.marshal()));
        for (auto& g : sp.witnesses) wit.append(P(g.marshal()));
        return py::make_tuple(P(sp.commitment.marshal()), cc, ys, wit);
      });
  m.def("write_commit_key", [](const std::string& path, size_t d, int64_t s) { write_commit_key(path, d, Scalar::from_i64(s)); },
        py::arg("path"), py::arg("d"), py::arg("secret") = 2);
  m.def("write_client_keys", [](const std::string& path, std::vector<std::pair<py::bytes, py::bytes>> keys) {
    std::vector<std::pair<Scalar, G1>> ks;
    for (auto& kv : keys) ks.push_back({Scalar::from_be(B(kv.first)), G1::unmarshal(B(kv.second))});
    write_client_keys(path, ks);
  });
  m.def("read_client_keys", [](const std::string& path) {
    py::list out;
    for (auto& kv : read_client_keys(path)) out.append(py::make_tuple(P(kv.first.to_be()), P(kv.second.marshal())));
    return out;
  });
  m.def("base64_encode", [](py::bytes b) { return base64_encode(B(b)); });
  m.def("base64_decode", [](const std::string& s) { return P(base64_decode(s)); });
  m.def("key_record_json", [](int64_t id, py::bytes pk, py::bytes sk) { return key_record_json({id, B(pk), B(sk)}); });

  // ---------------------------------------------------------------- shares (exact host reference)
  m.def("quantize", [](py::array_t<double, py::array::c_style | py::array::forcecast> v, int prec) {
    std::vector<double> x(v.data(), v.data() + v.size());
    auto q = quantize(x, prec);
    py::array_t<int64_t> out(py::ssize_t(q.size()));
    std::memcpy(out.mutable_data(), q.data(), q.size() * 8);
    return out;
  });
  m.def("chunk_stops", &chunk_stops);
  m.def("share_xs", &share_xs);
  m.def("poly_eval", [](std::vector<i64> c, i64 x) { return poly_eval(c.data(), int(c.size()), x); });
  m.def("poly_quotient", [](std::vector<i64> c, i64 x) { return poly_quotient(c.data(), int(c.size()), x); });
  m.def("recover_exact", [](std::vector<i64> xs, std::vector<i64> ys, int deg) -> py::object {
    std::vector<i64> out;
    if (!recover_exact(xs, ys, deg, &out)) return py::none();
    return py::cast(out);
  });
  m.def("recover_lstsq", &recover_lstsq);

  // ---------------------------------------------------------------- ledger
  py::class_<Update>(m, "Update")
      .def(py::init<>())
      .def_readwrite("source_id", &Update::source_id)
      .def_readwrite("iteration", &Update::iteration)
      .def_readwrite("delta", &Update::delta)
      .def_property("commitment", [](const Update& u) { return P(u.commitment); },
                    [](Update& u, py::bytes b) { u.commitment = B(b); })
      .def_readwrite("noise", &Update::noise)
      .def_readwrite("noised_delta", &Update::noised_delta)
      .def_readwrite("accepted", &Update::accepted)
      .def_property("signatures", [](const Update& u) {
        std::vector<py::bytes> r; for (auto& s : u.signatures) r.push_back(P(s)); return r;
      }, [](Update& u, std::vector<py::bytes> v) { u.signatures.clear(); for (auto& s : v) u.signatures.push_back(B(s)); })
      .def("__str__", &update_string);
  py::class_<BlockData>(m, "BlockData")
      .def(py::init<>())
      .def_readwrite("iteration", &BlockData::iteration)
      .def_property("global_w",
                    [](const BlockData& d) { return py::array_t<double>(py::ssize_t(d.global_w.size()), d.global_w.data()); },
                    [](BlockData& d, py::array_t<double, py::array::c_style | py::array::forcecast> a) {
                      d.global_w.assign(a.data(), a.data() + a.size());
                    })
      .def_readwrite("deltas", &BlockData::deltas)
      // `deltas` converts every Update (and its d-long vectors) into Python objects on each access
      .def_property_readonly("n_deltas", [](const BlockData& d) { return d.deltas.size(); })
      .def("gob", [](const BlockData& d) { return P(gob_encode_blockdata(d)); })
      .def("__str__", &blockdata_string);
  py::class_<Block>(m, "Block")
      .def(py::init<>())
      .def_readwrite("timestamp", &Block::timestamp)
      .def_readwrite("data", &Block::data)
      .def_property("prev_hash", [](const Block& b) { return P(b.prev_hash); }, [](Block& b, py::bytes x) { b.prev_hash = B(x); })
      .def_property("hash", [](const Block& b) { return P(b.hash); }, [](Block& b, py::bytes x) { b.hash = B(x); })
      .def_readwrite("stake", &Block::stake)
      .def("compute_hash", [](const Block& b) { return P(b.compute_hash()); })
      .def("set_hash", &Block::set_hash)
      .def("serialize", [](const Block& b) { return P(Blockchain::serialize_block(b)); })
      .def_static("deserialize", [](py::bytes x) {
        Bytes v = B(x);
        size_t used = 0;
        return Blockchain::deserialize_block(v.data(), v.size(), &used);
      });
  py::class_<Blockchain>(m, "Blockchain")
      .def_static("with_genesis", &Blockchain::with_genesis)
      .def_static("genesis", &Blockchain::genesis)
      .def_static("load", &Blockchain::load)
      .def_static("append_to_file", &Blockchain::append_to_file)
      .def("save", &Blockchain::save)
      .def("__len__", [](const Blockchain& c) { return c.blocks.size(); })
      .def("block", [](const Blockchain& c, size_t i) { return c.blocks.at(i); })
      .def("latest", [](const Blockchain& c) { return c.latest(); })
      // the latest block's hash alone (latest() copies the whole block, GlobalW included, into a new object)
      .def("latest_hash", [](const Blockchain& c) {
        const Bytes& h = c.latest().hash;
        return py::bytes(reinterpret_cast<const char*>(h.data()), h.size());
      })
      // the latest block's iteration alone (net/rpc answers it on every admitted call: no block copy)
      .def("latest_iteration", [](const Blockchain& c) { return c.latest().data.iteration; })
      .def("get", [](const Blockchain& c, i64 it) -> py::object {
        const Block* b = c.get(it);
        if (!b) return py::none();
        return py::cast(*b);
      })
      .def("add_block", &Blockchain::add_block)
      .def("append", &Blockchain::append)
      .def("verify", [](const Blockchain& c) {
        std::string why;
        bool ok = c.verify(&why);
        return py::make_tuple(ok, why);
      })
      .def("verify_range", [](const Blockchain& c, size_t from, size_t to) {
        std::string why;
        bool ok;
        {
          py::gil_scoped_release nogil;
          ok = c.verify_range(from, to, &why);
        }
        return py::make_tuple(ok, why);
      })
      .def("print_chain", &Blockchain::print_chain)
      .def("truncate", [](Blockchain& c, size_t n) { if (n < c.blocks.size()) c.blocks.resize(n); });
  m.def("gob_uint", [](uint64_t x) { Bytes b; gob_put_uint(b, x); return P(b); });
  m.def("gob_int", [](int64_t x) { Bytes b; gob_put_int(b, x); return P(b); });
  m.def("gob_float", [](double x) { Bytes b; gob_put_float(b, x); return P(b); });
  m.def("go_format_float", &go_format_float);

  // ---------------------------------------------------------------- protocol
  py::class_<ProtocolConfig>(m, "ProtocolConfig")
      .def(py::init<>())
      .def_readwrite("num_nodes", &ProtocolConfig::num_nodes)
      .def_readwrite("num_verifiers", &ProtocolConfig::num_verifiers)
      .def_readwrite("num_miners", &ProtocolConfig::num_miners)
      .def_readwrite("num_noisers", &ProtocolConfig::num_noisers)
      .def_readwrite("secure_agg", &ProtocolConfig::secure_agg)
      .def_readwrite("noising", &ProtocolConfig::noising)
      .def_readwrite("verification", &ProtocolConfig::verification)
      .def_readwrite("epsilon", &ProtocolConfig::epsilon)
      .def_readwrite("poisoning", &ProtocolConfig::poisoning)
      .def_readwrite("perc_samples", &ProtocolConfig::perc_samples)
      .def_readwrite("rand_sample", &ProtocolConfig::rand_sample)
      .def_readwrite("colluders", &ProtocolConfig::colluders)
      .def_readwrite("defense", &ProtocolConfig::defense)
      .def_readwrite("poly_size", &ProtocolConfig::poly_size)
      .def_readwrite("precision", &ProtocolConfig::precision)
      .def_readwrite("max_iterations", &ProtocolConfig::max_iterations)
      .def_readwrite("default_stake", &ProtocolConfig::default_stake)
      .def_readwrite("stake_unit", &ProtocolConfig::stake_unit)
      .def_readwrite("seed", &ProtocolConfig::seed)
      .def_readwrite("shared_inbox", &ProtocolConfig::shared_inbox)
      .def_readwrite("miner_cap", &ProtocolConfig::miner_cap)
      .def_readwrite("miner_block_div", &ProtocolConfig::miner_block_div)
      .def_readonly("num_samples", &ProtocolConfig::num_samples)
      .def_readonly("krum_thresh", &ProtocolConfig::krum_thresh)
      .def_readonly("total_shares", &ProtocolConfig::total_shares)
      .def_readonly("shares_per_miner", &ProtocolConfig::shares_per_miner)
      .def_readonly("miner_share_thresh", &ProtocolConfig::miner_share_thresh)
      .def_readonly("poisoning_index", &ProtocolConfig::poisoning_index)
      .def_readonly("collusion_thresh", &ProtocolConfig::collusion_thresh)
      .def("derive", &ProtocolConfig::derive);
  py::class_<RoundPlan>(m, "RoundPlan")
      .def_readonly("iteration", &RoundPlan::iteration)
      .def_readonly("verifiers", &RoundPlan::verifiers)
      .def_readonly("miners", &RoundPlan::miners)
      .def_readonly("workers", &RoundPlan::workers)
      .def_readonly("leader", &RoundPlan::leader)
      .def_readonly("live", &RoundPlan::live)
      .def_readonly("done", &RoundPlan::done);
  py::class_<RoundFSM::LeaderView>(m, "LeaderView")
      .def_readonly("leader_online", &RoundFSM::LeaderView::leader_online)
      .def_readonly("quorum", &RoundFSM::LeaderView::quorum)
      .def_readonly("node_list", &RoundFSM::LeaderView::node_list)
      .def_readonly("contributing_miners", &RoundFSM::LeaderView::contributing_miners);
  py::class_<RoundFSM>(m, "RoundFSM")
      .def(py::init<const ProtocolConfig&, i64>())
      .def_readonly("cfg", &RoundFSM::cfg)
      .def_readwrite("chain", &RoundFSM::chain)
      .def_readwrite("stake", &RoundFSM::stake)
      .def_readwrite("iteration", &RoundFSM::iteration)
      .def_readwrite("addresses", &RoundFSM::addresses)
      .def_readonly("plan", &RoundFSM::plan)
      .def("begin_round", &RoundFSM::begin_round, py::return_value_policy::copy)
      .def("verifier_inbox", &RoundFSM::verifier_inbox)
      .def("verifier_inboxes", &RoundFSM::verifier_inboxes)
      .def("leader_arrivals", &RoundFSM::leader_arrivals)
      .def("leader_cap", &RoundFSM::leader_cap)
      .def("leader_cap_size", &RoundFSM::leader_cap_size)
      .def("krum_clip", &RoundFSM::krum_clip)
      .def("approve", [](const RoundFSM& f, const std::map<i64, std::vector<i64>>& acc) {
        bool online = false;
        auto a = f.approve(acc, &online);
        return py::make_tuple(a, online);
      })
      .def("route_shares", &RoundFSM::route_shares)
      // the noiser lottery with this FSM's stake (no stake map round trip through a Python dict)
      .def("select_noisers_job", [](const RoundFSM& f, VrfJob& job, std::vector<i64> out_index,
                                    std::vector<i64> selfs, i64 nn, i64 n) {
        return select_noisers_impl(f.stake, job, std::move(out_index), std::move(selfs), nn, n);
      })
      // route_shares + leader_view without the routes crossing into Python: (leader_online, quorum,
      // node_list, contributing miners, {miner: share part of the node list's first worker})
      .def("route_view", [](const RoundFSM& f, const std::vector<i64>& approved) {
        auto routes = f.route_shares(approved);
        auto lv = f.leader_view(routes);
        py::dict part;
        if (!lv.node_list.empty())
          for (i64 m : lv.contributing_miners) {
            auto it = routes.find(m);
            if (it == routes.end()) continue;
            for (auto& wp : it->second)
              if (wp.first == lv.node_list[0]) {
                part[py::int_(m)] = py::int_(wp.second);
                break;
              }
          }
        return py::make_tuple(lv.leader_online, lv.quorum, lv.node_list, lv.contributing_miners, part);
      })
      .def("leader_view", &RoundFSM::leader_view)
      .def("route_updates", &RoundFSM::route_updates)
      .def("make_secagg_block", [](RoundFSM& f, py::array_t<double, py::array::c_style | py::array::forcecast> w,
                                   std::vector<i64> nodes, std::vector<py::bytes> comms, i64 now) {
        std::vector<Bytes> cs;
        cs.reserve(comms.size());
        for (auto& c : comms) cs.push_back(B(c));
        return f.make_secagg_block(w.data(), size_t(w.size()), nodes, std::move(cs), now);
      })
      // the same with the commitments as device-layout Jacobian rows (the pre-step's pinned read-back): only the
      // block's rows are marshalled (one inversion), in C++, on the round's block-build path
      .def("make_secagg_block_jac", [](RoundFSM& f, py::array_t<double, py::array::c_style | py::array::forcecast> w,
                                       std::vector<i64> nodes,
                                       py::array_t<uint32_t, py::array::c_style | py::array::forcecast> jac,
                                       std::vector<int64_t> rows, i64 now) {
        if (jac.ndim() != 2 || jac.shape(1) != 24) throw std::runtime_error("expected [n, 24] uint32");
        if (rows.size() != nodes.size()) throw std::runtime_error("rows/node_list mismatch");
        for (int64_t r : rows)
          if (r < 0 || r >= jac.shape(0)) throw std::runtime_error("commitment row out of range");
        std::vector<uint8_t> m(rows.size() * 64);
        marshal_jac_rows(jac.data(), rows.data(), rows.size(), m.data());
        std::vector<Bytes> cs(rows.size());
        for (size_t k = 0; k < rows.size(); ++k) cs[k].assign(m.begin() + 64 * k, m.begin() + 64 * (k + 1));
        return f.make_secagg_block(w.data(), size_t(w.size()), nodes, std::move(cs), now);
      })
      .def("make_plain_block", [](RoundFSM& f, py::array_t<double, py::array::c_style | py::array::forcecast> w,
                                  const std::vector<Update>& ups, i64 now) {
        return f.make_plain_block(std::vector<double>(w.data(), w.data() + w.size()), ups, now);
      })
      .def("make_plain_block_arrays",
           [](RoundFSM& f, py::array_t<double, py::array::c_style | py::array::forcecast> w0, std::vector<i64> ids,
              py::array_t<double, py::array::c_style | py::array::forcecast> deltas,
              py::array_t<double, py::array::c_style | py::array::forcecast> noised, std::vector<py::bytes> commits,
              std::vector<std::vector<py::bytes>> sigs, i64 now) {
             // plain-path block (honest.go:346-388) straight from [n, d] arrays: W = W0 + sum of the
             // deltas in `ids` order (float64), Update{delta, noise = noised - delta, noised_delta}
             const size_t n = ids.size(), d = size_t(w0.size());
             if (deltas.ndim() != 2 || size_t(deltas.shape(0)) != n || size_t(deltas.shape(1)) != d ||
                 noised.ndim() != 2 || size_t(noised.shape(0)) != n || size_t(noised.shape(1)) != d ||
                 commits.size() != n || sigs.size() != n)
               throw std::runtime_error("make_plain_block_arrays: shape mismatch");
             std::vector<double> W(w0.data(), w0.data() + d);
             std::vector<Update> ups(n);
             std::vector<Bytes> cm(n);
             std::vector<std::vector<Bytes>> sg(n);
             for (size_t k = 0; k < n; ++k) {
               cm[k] = B(commits[k]);
               for (auto& x : sigs[k]) sg[k].push_back(B(x));
             }
             {
               py::gil_scoped_release rel;
               for (size_t k = 0; k < n; ++k) {
                 const double* dv = deltas.data(py::ssize_t(k), 0);
                 const double* nv = noised.data(py::ssize_t(k), 0);
                 Update& u = ups[k];
                 u.source_id = ids[k];
                 u.iteration = f.iteration;
                 u.accepted = true;
                 u.delta.assign(dv, dv + d);
                 u.noised_delta.assign(nv, nv + d);
                 u.noise.resize(d);
                 for (size_t j = 0; j < d; ++j) {
                   u.noise[j] = nv[j] - dv[j];
                   W[j] += dv[j];
                 }
                 u.commitment = std::move(cm[k]);
                 u.signatures = std::move(sg[k]);
               }
             }
             return f.make_plain_block(W, ups, now);
           })
      .def("make_empty_block", &RoundFSM::make_empty_block)
      .def("commit_block", &RoundFSM::commit_block)
      .def("is_poisoner", &RoundFSM::is_poisoner, py::arg("id"), py::arg("fedsys") = false)
      .def("is_colluder", &RoundFSM::is_colluder)
      .def("round_seed", &RoundFSM::round_seed)
      .def("successor", &RoundFSM::successor)
      // The next round's speculative share plan in ONE call (head.py _spec_head_launch): the FSM as it will
      // be after committing `b`, every peer live -> (plan, every verifier's inbox, the leader's arrival
      // order, this rank's candidate workers [lo, hi) sorted by arrival, every candidate sorted), or None
      // when the run is over.  Candidates: every update some verifier judges, or every worker when
      // floor(nv/2) == 0 signatures suffice (main.go:1686).
      // horizon >= 0: only the first `horizon` candidates in the leader's arrival order are speculative rows (the
      // candidate list, this rank's rows and the Krum row map are cut to them); the tuple then ends with the full
      // candidate arrival order
      .def("spec_plan", [](RoundFSM& f, const Block& b, i64 lo, i64 hi, std::vector<i64> xrow, i64 U,
                           i64 horizon) -> py::object {
        RoundFSM s = f.successor(b);
        const i64 n = s.cfg.num_nodes;
        std::vector<u8> live(size_t(n), 1);
        const RoundPlan plan = s.begin_round(live);
        if (plan.done) return py::none();
        auto inboxes = s.verifier_inboxes(plan.workers);
        std::vector<u8> cand(size_t(n), 0);
        if (plan.verifiers.size() / 2 == 0) {
          for (i64 w : plan.workers) cand.at(size_t(w)) = 1;
        } else {
          for (auto& ib : inboxes)
            for (i64 w : ib) cand.at(size_t(w)) = 1;
        }
        auto arrivals = s.leader_arrivals();
        std::vector<i64> rank(size_t(n), i64(1) << 30);
        for (size_t i = 0; i < arrivals.size(); ++i) rank.at(size_t(arrivals[i])) = i64(i);
        std::vector<i64> order;   // the candidates in the leader's arrival order
        for (i64 w : arrivals)
          if (cand.at(size_t(w))) order.push_back(w);
        if (horizon >= 0 && horizon < i64(order.size()))
          for (size_t i = size_t(horizon); i < order.size(); ++i) cand[size_t(order[i])] = 0;
        std::vector<i64> spec, cands;
        for (i64 w : plan.workers)
          if (cand.at(size_t(w)) && w >= lo && w < hi) spec.push_back(w);
        std::stable_sort(spec.begin(), spec.end(), [&](i64 a, i64 c) { return rank[size_t(a)] < rank[size_t(c)]; });
        for (i64 w = 0; w < n; ++w)
          if (cand[size_t(w)]) cands.push_back(w);
        if (xrow.empty()) return py::make_tuple(plan, inboxes, arrivals, spec, cands, order);
        // Krum's static tables for this plan (verify.py _krum_static): every verifier's inbox as rows of the
        // selection input (xrow: peer -> row, -1 none), each row's leader-arrival rank, speculative row -> row
        if (xrow.size() != size_t(n)) throw std::runtime_error("spec_plan: xrow must map every peer");
        const size_t ni = inboxes.empty() ? 0 : inboxes[0].size();
        py::array_t<int32_t> inbox({py::ssize_t(inboxes.size()), py::ssize_t(ni)});
        int32_t* ib = inbox.mutable_data();
        for (size_t v = 0; v < inboxes.size(); ++v) {
          if (inboxes[v].size() != ni) throw std::runtime_error("spec_plan: ragged inboxes");
          for (size_t j = 0; j < ni; ++j) ib[v * ni + j] = int32_t(xrow.at(size_t(inboxes[v][j])));
        }
        py::array_t<int32_t> rk(U > 0 ? U : 0);
        int32_t* r = rk.mutable_data();
        for (i64 u = 0; u < U; ++u) r[u] = -1;
        for (size_t i = 0; i < arrivals.size(); ++i) {
          const i64 x = xrow.at(size_t(arrivals[i]));
          if (x >= 0 && x < U) r[x] = int32_t(i);
        }
        py::array_t<int32_t> src(py::ssize_t(spec.size()));
        int32_t* sr = src.mutable_data();
        for (size_t i = 0; i < spec.size(); ++i) sr[i] = int32_t(xrow.at(size_t(spec[i])));
        return py::make_tuple(plan, inboxes, arrivals, spec, cands, inbox, rk, src, order);
      }, py::arg("block"), py::arg("lo"), py::arg("hi"), py::arg("xrow") = std::vector<i64>{}, py::arg("U") = 0,
         py::arg("horizon") = -1);
  m.def("select_roles", [](const std::map<i64, i64>& stake, py::bytes h, i64 nv, i64 na, i64 n) {
    std::vector<i64> v, mm;
    select_roles(stake, B(h), nv, na, n, &v, &mm);
    return py::make_tuple(v, mm);
  });
  m.def("select_noisers", [](const std::map<i64, i64>& stake, py::bytes out, i64 self, i64 nn, i64 n) {
    return select_noisers(stake, B(out), self, nn, n);
  });
  m.def("select_noisers_batch", [](const std::map<i64, i64>& stake, std::vector<py::bytes> outs,
                                   std::vector<i64> selfs, i64 nn, i64 n) {
    if (outs.size() != selfs.size()) throw std::runtime_error("outs/selfs length mismatch");
    std::vector<std::vector<i64>> r;
    r.reserve(outs.size());
    const Lottery table(stake, n, Bytes{});
    for (size_t k = 0; k < outs.size(); ++k) r.push_back(select_noisers(table, B(outs[k]), selfs[k], nn));
    return r;
  });
  // every worker's noisers straight from a VRF batch's outputs (no Python bytes in between): waits
  // for the outputs only; out_index[k] = the job's output of worker selfs[k] (empty: k itself).
  // Returns int64 [len(selfs), nn].  Same draws as select_noisers (equivalence-tested).
  m.def("select_noisers_job", [](const std::map<i64, i64>& stake, VrfJob& job, std::vector<i64> out_index,
                                 std::vector<i64> selfs, i64 nn, i64 n) {
    return select_noisers_impl(stake, job, std::move(out_index), std::move(selfs), nn, n);
  });
  // the lottery with the stake a block will leave the FSM with (commit_block: the block's map when it carries
  // one) -- the speculative front draws the next round's noisers before the block is committed
  m.def("select_noisers_job_after", [](const RoundFSM& f, const Block& b, VrfJob& job, std::vector<i64> out_index,
                                       std::vector<i64> selfs, i64 nn, i64 n) {
    return select_noisers_impl(b.stake.empty() ? f.stake : b.stake, job, std::move(out_index), std::move(selfs), nn, n);
  });
  m.def("krum_scores", [](py::array_t<double, py::array::c_style | py::array::forcecast> X, i64 groupsize) {
    if (X.ndim() != 2) throw std::runtime_error("X must be 2-D");
    return krum_scores(X.data(), X.shape(0), X.shape(1), groupsize);
  });
  m.def("krum_select", &krum_select);
  m.def("seeded_permutation", &seeded_permutation);
  py::class_<FedSysConfig>(m, "FedSysConfig")
      .def(py::init<>())
      .def_readwrite("num_nodes", &FedSysConfig::num_nodes)
      .def_readwrite("perc_samples", &FedSysConfig::perc_samples)
      .def_readwrite("rand_sample", &FedSysConfig::rand_sample)
      .def_readwrite("poisoning", &FedSysConfig::poisoning)
      .def_readonly("num_samples", &FedSysConfig::num_samples)
      .def_readonly("random_samples", &FedSysConfig::random_samples)
      .def("derive", &FedSysConfig::derive);
  m.def("fedsys_select", &fedsys_select);
}
