// Wave issue priority of the round's kernels (s_setprio).  On CDNA4 a SIMD arbitrates VALU issue between its
// resident waves by priority, then by age (MI355X_MICROARCH.md, two waves per SIMD), and kernels of the
// round's streams share SIMDs: at equal priority the OLDER waves win, so work launched first (the pre-step's
// commitment MSM, the witness sums) took issue slots from the speculative share MSM that the round's recovery
// waits for.  Stream priorities order only workgroup dispatch, not issue.  Classes:
#pragma once
#define BSC_PRIO_CRITICAL 3   // the round's latency chains: Krum scores / vote, selection flags, recovery, audit,
                              // the full commitments' sums
#define BSC_PRIO_SPEC 2       // the speculative share MSM (gates the recovery)
#define BSC_PRIO_AHEAD 1      // needed later in the round: the pre-step's commitment MSM (the block), evaluation,
                              // early commitment sums
// 0 (the hardware default): background -- the miners' witness sums (no consumer in the round), batched VRF
// proofs (the run's final flush: CRITICAL), KZG audit sums.
// The argument must be a constant; call it before the kernel's main work, under a wave-uniform condition (a
// kernel argument) if any, since s_setprio is a scalar instruction.
//
// The classes apply to one rank per process driving its GPU alone (bsc_wave_prio(1), the default).  With
// several ranks the engine turns them off (bsc_wave_prio(0)): RCCL's collective kernels run at the default
// priority and spin on their peers' flags, and under prio-2 share MSMs of two ranks sharing a GPU a collective
// stalled for 0.1-0.3 s (2-rank RCCL rehearsal).  Each kernel file holds its own flag (one per translation
// unit, named by BSC_PRIO_FLAG before the include) and exports its setter; kernels read it once,
// wave-uniformly.  The flag has external linkage on purpose: a `static` __device__ variable that the host
// addresses is externalised with default visibility and read through the GOT (two dependent scalar loads at
// every kernel's entry); a plain one is protected and costs one PC-relative load.
#ifndef BSC_PRIO_FLAG
#error "define BSC_PRIO_FLAG (a per-file name) before including wave_prio.h"
#endif
__device__ int BSC_PRIO_FLAG = 1;
#define BSC_SET_PRIO(p)                                  \
  do {                                                   \
    if (BSC_PRIO_FLAG) __builtin_amdgcn_s_setprio(p);    \
  } while (0)
#define BSC_PRIO_SETTER(name)                                                                        \
  extern "C" int name(int on) {                                                                      \
    return (int)hipMemcpyToSymbol(HIP_SYMBOL(BSC_PRIO_FLAG), &on, sizeof(int), 0, hipMemcpyHostToDevice); \
  }
