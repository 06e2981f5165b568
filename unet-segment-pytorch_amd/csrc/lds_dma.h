// lds_dma.h — LDS-DMA plumbing shared by the operand-pipelined kernels (conv5.hip, wgrad5.hip): raw buffer
// resources as SGPR quads, buffer_load ... lds issued as inline asm, hand-counted vmcnt waits and a workgroup
// barrier that leaves the DMA queue alone.
#pragma once
#include "conv_common.h"

namespace unet {

typedef __attribute__((address_space(3))) const void* lds_ptr_t;
typedef __attribute__((ext_vector_type(4))) unsigned rsrc4_t;   // buffer resource as an SGPR quad

// raw buffer resource (range = bytes, OOB loads return 0) for the inline-asm DMAs below
__device__ __forceinline__ rsrc4_t mk_rsrc4(const void* p, unsigned bytes) {
  const unsigned long long a = (unsigned long long)p;
  rsrc4_t r;
  r.x = __builtin_amdgcn_readfirstlane((unsigned)a);
  r.y = __builtin_amdgcn_readfirstlane((unsigned)(a >> 32) & 0xffffu);
  r.z = __builtin_amdgcn_readfirstlane(bytes);
  r.w = 0x00020000u;
  return r;
}

// LDS DMA (buffer_load ... lds: M0 = wave-uniform LDS base, lane l lands at base + l * size).  Issued as
// inline asm on purpose: the compiler's waitcnt pass treats every LDS read that may alias an outstanding
// LDS-DMA write as dependent on it and puts s_waitcnt vmcnt(0) in front of it — which drains the two-chunk
// prefetch on every chunk.  The kernel orders its DMAs itself (wait_vm per chunk + lds_barrier); the asm's
// memory clobber keeps the compiler from moving LDS accesses across the issue.  The s_nop 4 supplies the
// wait states the compiler's hazard recognizer inserts for the builtin but cannot see inside an asm
// statement: 5 between a VALU write of an SGPR (v_readlane of a resource spilled to VGPR lanes,
// v_readfirstlane) and a VMEM instruction reading it, 1 between an SALU write of M0 and an LDS DMA.
__device__ __forceinline__ unsigned lds_addr(const void* lds) {
  return __builtin_amdgcn_readfirstlane((unsigned)(unsigned long long)(lds_ptr_t)lds);
}
// m0: the wave-uniform LDS byte address (an SGPR value)
__device__ __forceinline__ void dma16(rsrc4_t r, unsigned m0, unsigned voff) {
  asm volatile("s_nop 4\n\tbuffer_load_dwordx4 %0, %1, 0 offen lds" ::"v"(voff), "s"(r), "{m0}"(m0) : "memory");
}
__device__ __forceinline__ void dma4(rsrc4_t r, unsigned m0, unsigned voff) {
  asm volatile("s_nop 4\n\tbuffer_load_dword %0, %1, 0 offen lds" ::"v"(voff), "s"(r), "{m0}"(m0) : "memory");
}

// s_waitcnt vmcnt(N), nothing else; asm with a memory clobber so no LDS read is hoisted above it
template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
// workgroup barrier that leaves the DMA queue alone: this wave's LDS writes done, then s_barrier
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

}  // namespace unet
