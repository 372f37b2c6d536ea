// The verification all_gather of several ranks (one rank per GPU), packed and unpacked in one kernel each.
//
// Every rank contributes ONE row of a resident [world, row_bytes] buffer and the caller all_gathers it in place
// (RCCL: sendbuff = recvbuff + rank * count):
//
//   row = [ split Gram slot : chunk x 256 f64 ][ commitments : maxlocal x pw u32 ][ noiser ids : maxlocal x nn
//          i32 ][ noiser weights : maxlocal x nn f32 ]   (16-byte padded; the Gram slot is written by the Gram
//          kernel itself, bsc_gram_stacked_range with its output pointed here)
//
// bsc_vg_pack   -- this rank's commitment rows (from the pre-step's rows through a slot map) and its workers'
//                  noiser ids / weights (passed by value in the kernel's arguments: no upload) into its row
// bsc_vg_unpack -- after the gather: the whole tiled Gram [npairs, 256] (rank r's slot holds pairs
//                  [r chunk, (r + 1) chunk)), the flat [world maxlocal, nn] noiser ids / weights, and the
//                  round's workers' commitment rows straight into pinned host memory (worker flat rows in the
//                  kernel's arguments)
//
// They replace ~15 tensor operations of the Python path (zero fills, index copies, a concatenation, per-part
// slicing copies and uploads) on the round's host thread.  Reference: the per-worker commitments and noise a
// verifier receives (DistSys/main.go:1513-1589, krum.go:227-365).
#include <hip/hip_runtime.h>
#include <stdint.h>

#define VG_MAX_SLOTS 128   // local peer slots per rank
#define VG_MAX_NZ 256      // maxlocal x nn noiser entries per rank
#define VG_MAX_WORKERS 1024 // workers whose commitment rows are read back (weak scaling: 800 peers)

struct VgPackArgs {
  int src_row[VG_MAX_SLOTS];   // slot j (local peer lo + j) -> row of the commitment source, -1: zeros
  int nz[VG_MAX_NZ];
  float sc[VG_MAX_NZ];
};

struct VgUnpackArgs {
  int wrow[VG_MAX_WORKERS];    // flat rows (rank * maxlocal + slot) of the round's workers, plan order
};

extern "C" __global__ void __launch_bounds__(256) k_vg_pack(uint8_t* row, long long commit_off, long long nz_off,
                                                           long long sc_off, const uint32_t* commits, int maxlocal,
                                                           int pw, int nnz, VgPackArgs a) {
  uint32_t* dc = (uint32_t*)(row + commit_off);
  const int nc = maxlocal * pw;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < nc + 2 * nnz; i += gridDim.x * blockDim.x) {
    if (i < nc) {
      const int j = i / pw, c = i - j * pw;
      const int s = a.src_row[j];
      dc[i] = s >= 0 ? commits[(size_t)s * pw + c] : 0u;
    } else if (i < nc + nnz) {
      ((int*)(row + nz_off))[i - nc] = a.nz[i - nc];
    } else {
      ((float*)(row + sc_off))[i - nc - nnz] = a.sc[i - nc - nnz];
    }
  }
}

extern "C" __global__ void __launch_bounds__(256) k_vg_unpack(const uint8_t* recv, long long row_bytes, int chunk,
                                                             int npairs, long long commit_off, long long nz_off,
                                                             long long sc_off, int maxlocal, int pw, int nn,
                                                             int world, int nw, double* gram, int* nz, float* sc,
                                                             uint32_t* commits_host, VgUnpackArgs a) {
  const long long ng = (long long)npairs * 256, nzn = (long long)world * maxlocal * nn, nc = (long long)nw * pw;
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < ng) {
    const int p = (int)(i >> 8), e = (int)(i & 255);
    const int r = p / chunk, lp = p - r * chunk;
    gram[i] = ((const double*)(recv + (size_t)r * row_bytes))[(size_t)lp * 256 + e];
  } else if (i < ng + nzn) {
    const long long k = i - ng;
    const int row = (int)(k / nn), s = (int)(k - (long long)row * nn);
    const int r = row / maxlocal, j = row - r * maxlocal;
    const uint8_t* src = recv + (size_t)r * row_bytes;
    nz[k] = ((const int*)(src + nz_off))[j * nn + s];
    sc[k] = ((const float*)(src + sc_off))[j * nn + s];
  } else if (i < ng + nzn + nc) {
    const long long k = i - ng - nzn;
    const int w = (int)(k / pw), c = (int)(k - (long long)w * pw);
    const int f = a.wrow[w];
    const int r = f / maxlocal, j = f - r * maxlocal;
    commits_host[k] = ((const uint32_t*)(recv + (size_t)r * row_bytes + commit_off))[(size_t)j * pw + c];
  }
}

extern "C" int bsc_vg_limits(int* out) {
  out[0] = VG_MAX_SLOTS;
  out[1] = VG_MAX_NZ;
  out[2] = VG_MAX_WORKERS;
  return 0;
}

extern "C" int bsc_vg_pack(uint8_t* row, long long commit_off, long long nz_off, long long sc_off,
                           const uint32_t* commits, int maxlocal, int pw, const int* src_row, const int* nz,
                           const float* sc, int nnz, void* stream) {
  if (maxlocal > VG_MAX_SLOTS || nnz > VG_MAX_NZ || maxlocal <= 0 || pw <= 0 || nnz < 0) return -1;
  VgPackArgs a;
  for (int j = 0; j < VG_MAX_SLOTS; ++j) a.src_row[j] = j < maxlocal ? src_row[j] : -1;
  for (int k = 0; k < VG_MAX_NZ; ++k) {
    a.nz[k] = k < nnz ? nz[k] : 0;
    a.sc[k] = k < nnz ? sc[k] : 0.0f;
  }
  const int n = maxlocal * pw + 2 * nnz;
  hipLaunchKernelGGL(k_vg_pack, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, row, commit_off, nz_off,
                     sc_off, commits, maxlocal, pw, nnz, a);
  return (int)hipGetLastError();
}

extern "C" int bsc_vg_unpack(const uint8_t* recv, long long row_bytes, int chunk, int npairs, long long commit_off,
                             long long nz_off, long long sc_off, int maxlocal, int pw, int nn, int world,
                             const int* wrow, int nw, double* gram, int* nz, float* sc, uint32_t* commits_host,
                             void* stream) {
  if (nw > VG_MAX_WORKERS || nw < 0 || maxlocal <= 0 || world <= 0 || (npairs > 0 && chunk <= 0)) return -1;
  VgUnpackArgs a;
  for (int k = 0; k < VG_MAX_WORKERS; ++k) {
    const int f = k < nw ? wrow[k] : 0;
    if (f < 0 || f >= world * maxlocal) return -2;   // a row outside the gathered buffer
    a.wrow[k] = f;
  }
  const long long total = (long long)npairs * 256 + (long long)world * maxlocal * nn + (long long)nw * pw;
  if (total == 0) return 0;
  hipLaunchKernelGGL(k_vg_unpack, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, (hipStream_t)stream, recv,
                     row_bytes, chunk, npairs, commit_off, nz_off, sc_off, maxlocal, pw, nn, world, nw, gram, nz, sc,
                     commits_host, a);
  return (int)hipGetLastError();
}
