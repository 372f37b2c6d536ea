// Wave issue priority of the round's kernels (s_setprio).  On CDNA4 a SIMD arbitrates VALU issue between its
// resident waves by priority, then by age (MI355X_MICROARCH.md, two waves per SIMD), and kernels of the
// round's streams share SIMDs: at equal priority the OLDER waves win, so work launched first (the pre-step's
// commitment MSM, the witness sums) took issue slots from the speculative share MSM that the round's recovery
// waits for.  Stream priorities order only workgroup dispatch, not issue.  Classes:
#pragma once
#define BSC_PRIO_CRITICAL 3   // the round's latency chains: Krum scores / vote, selection flags, recovery, audit,
                              // the full commitments' sums
#define BSC_PRIO_SPEC 2       // the share MSMs: speculative (gates the recovery), pre-step commitments (the block)
#define BSC_PRIO_AHEAD 1      // needed later in the round: Gram, evaluation, pre-step step, early commitment sums
// 0 (the hardware default): background -- the miners' witness sums (no consumer in the round), batched VRF
// proofs (the run's final flush: CRITICAL), KZG audit sums.
// The argument must be a constant; call it before the kernel's main work, under a wave-uniform condition (a
// kernel argument) if any, since s_setprio is a scalar instruction.
#define BSC_SET_PRIO(p) __builtin_amdgcn_s_setprio(p)
