// lat_probe.hip -- per-instruction-class latencies of ONE wave alone on a SIMD
// (gfx950), the inputs of the C3 latency-floor model.
// Diagnostics only: built by `hipcc --offload-arch=gfx950 -O2 -o build/live/lat_probe tools/lat_probe.hip`, never
// linked into the library.  Each probe runs a chain of dependent instructions
// (inline asm, so the compiler adds nothing between them), timed with
// s_memtime (shader clock), and prints cycles per link.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

constexpr int kReps = 64;  // chain links per asm block: 16, run kReps times

#define TIMED(body)                                                                  \
  uint64_t t0 = __builtin_amdgcn_s_memtime();                                        \
  for (int rep = 0; rep < kReps; ++rep) {                                            \
    body                                                                             \
  }                                                                                  \
  uint64_t t1 = __builtin_amdgcn_s_memtime();

#define X4(s) s s s s
#define X16(s) X4(s) X4(s) X4(s) X4(s)

// 0: dependent v_add_u32 (32-bit VALU)
// 1: dependent v_lshl_add_u64 (64-bit VALU add)
// 2: dependent v_add_co_u32 + v_addc_co_u32 (the 64-bit add pair: 2 instructions per link)
// 3: eight independent v_add_u32 chains interleaved (issue cost per instruction)
// 4: DPP: s_nop 1 + v_add_u32_dpp row_shr:1 (dependent; the nop is the DPP read hazard)
// 5: v_readlane_b32 -> s_add_u32 -> v_mov_b32 (VALU -> SGPR -> VALU round trip, 3 instructions per link)
// 6: v_cmp_eq_u32 vcc + s_cbranch_vccz (a ballot-and-branch, taken to the next instruction)
// 7: dependent s_add_u32 (SALU)
// 8: ds_read_b32 pointer chase in LDS (address = previous result)
// 9: global_store_dword + s_waitcnt vmcnt(0) (one store's acknowledgement)
// 10: v_cmp_lt_u32 vcc + v_cndmask_b32 (a select/min link, 2 instructions)
// 11: s_setprio-free uniform branch ladder: s_cmp_lt_u32 + s_cbranch_scc1 (not taken)
__global__ void probe(int which, uint64_t* out, uint32_t* gbuf) {
  __shared__ uint32_t lds[64];
  const int lane = threadIdx.x;
  lds[lane] = 0;  // pointer chase: every slot points at slot 0 (address 0)
  __syncthreads();
  uint32_t v = lane, w = 1;
  uint64_t v64 = lane, w64 = 3;
  uint32_t s = 0;
  uint64_t cyc = 0;
  switch (which) {
    case 0: { TIMED(asm volatile(X16("v_add_u32 %0, %0, %1\n\t") : "+v"(v) : "v"(w));) cyc = t1 - t0; break; }
    case 1: { TIMED(asm volatile(X16("v_lshl_add_u64 %0, %0, 0, %1\n\t") : "+v"(v64) : "v"(w64));) cyc = t1 - t0; break; }
    case 2: {
      uint32_t lo = lane, hi = 0;
      TIMED(asm volatile(X16("v_add_co_u32 %0, vcc, %0, %2\n\tv_addc_co_u32 %1, vcc, %1, %2, vcc\n\t")
                         : "+v"(lo), "+v"(hi) : "v"(w) : "vcc");)
      cyc = t1 - t0;
      v = lo ^ hi;
      break;
    }
    case 3: {
      uint32_t a0 = lane, a1 = lane, a2 = lane, a3 = lane, a4 = lane, a5 = lane, a6 = lane, a7 = lane;
      TIMED(asm volatile(X4("v_add_u32 %0, %0, %8\n\tv_add_u32 %1, %1, %8\n\tv_add_u32 %2, %2, %8\n\tv_add_u32 %3, %3, %8\n\t"
                            "v_add_u32 %4, %4, %8\n\tv_add_u32 %5, %5, %8\n\tv_add_u32 %6, %6, %8\n\tv_add_u32 %7, %7, %8\n\t")
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                         : "v"(w));)
      cyc = (t1 - t0) / 2;  // 32 instructions per block: per 16 for the common divisor below
      v = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
      break;
    }
    case 4: { TIMED(asm volatile(X16("s_nop 1\n\tv_add_u32_dpp %0, %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf\n\t") : "+v"(v));) cyc = t1 - t0; break; }
    case 5: {
      TIMED(asm volatile(X16("v_readlane_b32 %1, %0, 0\n\ts_add_u32 %1, %1, 1\n\tv_mov_b32 %0, %1\n\t") : "+v"(v), "+s"(s) : : "scc");)
      cyc = t1 - t0;
      break;
    }
    case 6: {
      TIMED(asm volatile(X16("v_cmp_eq_u32 vcc, %0, %1\n\ts_cbranch_vccz 1f\n1:\n\t") : : "v"(v), "v"(w) : "vcc");)
      cyc = t1 - t0;
      break;
    }
    case 7: { TIMED(asm volatile(X16("s_add_u32 %0, %0, 1\n\t") : "+s"(s) : : "scc");) cyc = t1 - t0; break; }
    case 8: {
      uint32_t p = 0;
      TIMED(asm volatile(X16("ds_read_b32 %0, %0\n\ts_waitcnt lgkmcnt(0)\n\t") : "+v"(p) : : "memory");)
      cyc = t1 - t0;
      v = p;
      break;
    }
    case 9: {
      uint32_t* dst = gbuf + lane;
      TIMED(asm volatile(X16("global_store_dword %0, %1, off\n\ts_waitcnt vmcnt(0)\n\t") : : "v"(dst), "v"(v) : "memory");)
      cyc = t1 - t0;
      break;
    }
    case 10: {
      TIMED(asm volatile(X16("v_cmp_lt_u32 vcc, %0, %1\n\tv_cndmask_b32 %0, %1, %0, vcc\n\t") : "+v"(v) : "v"(w) : "vcc");)
      cyc = t1 - t0;
      break;
    }
    default: {
      TIMED(asm volatile(X16("s_cmp_lt_u32 %0, 0\n\ts_cbranch_scc1 1f\n1:\n\t") : : "s"(s) : "scc");)
      cyc = t1 - t0;
      break;
    }
  }
  if (lane == 0) {
    out[0] = cyc;
    out[1] = (uint64_t)v + v64 + s;  // keep the chains live
  }
}

int main() {
  const char* names[] = {"valu_add_u32_dep",   "valu_lshl_add_u64_dep", "valu_add64_pair_dep(2 instr)",
                         "valu_add_u32_indep", "dpp_row_shr_dep(+s_nop 1)", "readlane_salu_vmov(3 instr)",
                         "vcmp_vcc_cbranch(2 instr)", "salu_add_dep", "ds_read_b32_chase", "store_vmcnt0",
                         "cmp_cndmask(2 instr)", "scmp_cbranch_not_taken(2 instr)"};
  uint64_t* d_out;
  uint32_t* d_buf;
  if (hipMalloc(&d_out, 16) != hipSuccess || hipMalloc(&d_buf, 4096) != hipSuccess) return 1;
  printf("{\n");
  for (int i = 0; i < 12; ++i) {
    uint64_t h[2] = {0, 0};
    for (int warm = 0; warm < 2; ++warm) {  // the second launch is the one reported
      hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, i, d_out, d_buf);
      if (hipDeviceSynchronize() != hipSuccess) return 2;
    }
    if (hipMemcpy(h, d_out, 16, hipMemcpyDeviceToHost) != hipSuccess) return 3;
    printf("  \"%s\": %.2f%s\n", names[i], (double)h[0] / (16.0 * kReps), i + 1 < 12 ? "," : "");
  }
  printf("}\n");
  return 0;
}
