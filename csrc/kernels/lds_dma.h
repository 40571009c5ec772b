// LDS-DMA helpers shared by the LDS-staged gradient kernels (grad_dense.hip, grad_mfma.hip).
#pragma once

#include "common.h"

namespace eh {

// The LDS-DMA loads (global_load_lds, 16-byte and 4-byte pieces) are issued by inline asm: through
// the builtin, hipcc cannot tell the stage being filled from the one being read and waits vmcnt(0)
// before every ds_read, which drains the prefetch (checked in the .s).  The kernels count and wait
// for their own loads instead: "stage t landed" is vmcnt <= the loads this wave issued for the
// stages after t (tests/test_isa_checks.py checks the compiler adds no loads of its own inside the
// counted stage loop; -DEH_FULL_VMCNT turns every such wait into vmcnt(0) for a suspected LDS race).
// glds16 carries the X stream: nt, like kStreamAux (common.h); glds4 (labels) keeps the default policy.
__device__ __forceinline__ void glds16(const void* g, unsigned lds) {
  int keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(g), "s"(lds) : "memory");
}
__device__ __forceinline__ void glds4(const void* g, unsigned lds) {
  int keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(g), "s"(lds) : "memory");
}
// s_waitcnt vmcnt(n) for a wave-uniform runtime n (the immediate must be a constant; n > 63 waits
// for 63, which is stricter and therefore safe).
__device__ __forceinline__ void wait_vmcnt(int n) {
#ifdef EH_FULL_VMCNT
  n = 0;  // debug build: every stage wait drains all loads
#endif
  // The two-stage ring (the default) always waits for everything: test that first.  Testing a
  // readfirstlane copy keeps the compiler from folding it into the switch's compare tree.
  if (__builtin_amdgcn_readfirstlane(n) <= 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    return;
  }
  switch (n) {
#define EH_W(k) case k: asm volatile("s_waitcnt vmcnt(" #k ")" ::: "memory"); return;
#define EH_W8(k) EH_W(k) EH_W(k + 1) EH_W(k + 2) EH_W(k + 3) EH_W(k + 4) EH_W(k + 5) EH_W(k + 6) EH_W(k + 7)
    EH_W8(0) EH_W8(8) EH_W8(16) EH_W8(24) EH_W8(32) EH_W8(40) EH_W8(48) EH_W8(56)
#undef EH_W8
#undef EH_W
    default: asm volatile("s_waitcnt vmcnt(63)" ::: "memory");
  }
}


}  // namespace eh
