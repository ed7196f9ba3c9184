// XCD (accelerator complex die) of the executing wave on MI355X: HW_REG_XCC_ID[3:0]. 8 XCDs, each with its own
// L2; workgroups are dispatched round-robin over them (blockIdx % 8), which kernels may exploit for locality but
// must not rely on for correctness.
#pragma once
#include <hip/hip_runtime.h>

__device__ __forceinline__ int mifx_xcc_id() {
  int v;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
  return v & 15;
}
