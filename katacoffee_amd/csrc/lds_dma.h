// LDS-DMA helpers shared by the network kernels (nn.hip, nn_layered.hip): weight
// streams land in LDS through global_load_lds_dwordx4 (no VGPR destination) and are
// published by a counted vmcnt wait plus a barrier that keeps other DMA in flight.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "kc_common.h"

namespace kc {

// LDS byte address of a pointer into dynamic shared memory.
KC_D uint32_t ldsAddr(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}

// One 1-KiB LDS-DMA piece: each lane's 16 bytes at src land at lds + 16 * lane
// (global_load_lds_dwordx4, no VGPR destination).  Issued from inline asm so the
// compiler neither waits on it nor reorders LDS accesses around it; completion is
// counted by hand (s_waitcnt vmcnt) before the barrier that publishes the slot.
KC_D void glds16(const void* src, uint32_t lds) {
  const uint32_t dst = __builtin_amdgcn_readfirstlane(lds);
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(src), "s"(dst)
               : "memory");
}

// The same piece addressed as a wave-uniform base (SGPR pair, global_load's saddr form)
// plus a 32-bit per-lane byte offset: a burst of pieces costs no VGPR per piece (the
// per-lane 64-bit addresses of glds16 raise the network kernels' VGPR allocation,
// which decides whether the other game group's search waves fit beside them on a CU).
KC_D void glds16s(const void* base, uint32_t laneOff, uint32_t lds) {
  const uint32_t dst = __builtin_amdgcn_readfirstlane(lds);
  // (readfirstlane returns int: widen through uint32_t, a sign extension of the low
  // word would corrupt the high word of addresses with bit 31 set)
  const uint64_t b = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)base) |
                     ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)((uintptr_t)base >> 32)) << 32);
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(laneOff), "s"(b), "s"(dst)
               : "memory");
}

template <int N>
KC_D void waitVm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
// Workgroup barrier that leaves LDS-DMA loads in flight (a __syncthreads()
// would drain them with vmcnt(0)); LDS reads and writes issued before it complete.
KC_D void barrierKeepDma() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

}  // namespace kc
