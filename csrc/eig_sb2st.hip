// Stage 2 of the two-stage symmetric eigensolver: band (half-bandwidth 16)
// -> tridiagonal by bulge chasing (reference semantics
// kfac/layers/utils.py:45-74).  Stage 1 is csrc/eig_sy2sb.hip; the exact
// operation order is modelled in fp64 by scripts/models/two_stage_model.py
// (sb2st).
//
//   task (s, j):  c = s (j = 0) or s + 1 + (j-1) 16, rows I = r0 .. r1 with
//                 r0 = s + 1 + 16 j, r1 = min(r0 + 15, n - 1); Householder
//                 reflector from B[I, c]; B <- H B H on the stored lower band:
//                 column c, the left block B[I, c+1 .. r0-1], the diagonal
//                 block B[I, I] (both sides), the block below
//                 B[r1+1 .. r1+16, I] (the next bulge).
//   (s+1, j) may run once (s, j+2) is done.
//
// Band storage: row r holds B[r][r-31 .. r] (32 floats, row-major, rows n ..
// n + 31 zero); a task touches the 32 rows r0 .. r0 + 31 only.
//
// MI355X mapping: a pipeline of 4-wave workgroups per matrix.  Workgroup g
// runs the 4 consecutive sweeps 4g .. 4g+3 ("a group"), one per wave, in
// lockstep ticks -- wave w runs task t - 3 w at tick t, one LDS barrier per
// tick:
//   * each wave keeps a 4-block ring of 16-row band blocks in LDS (block k =
//     rows s+1+16k .. s+16+16k of its sweep); task j works on blocks j, j+1
//     and fills block j+1 from the previous wave's ring (its blocks j+1 and
//     j+2, one row shifted), which that wave finished in earlier ticks;
//   * wave 0 reads its blocks from the band in global memory, two blocks
//     every other tick, up to five blocks ahead, after polling the previous
//     workgroup's published block count;
//   * wave 3 writes each finished block back (sc1 write-through stores) and
//     publishes its count two ticks later, after its own vmcnt wait (the
//     guide's sc1-granule hand-off form: stores and loads all sc1, one
//     publishing wave, one workgroup per CU); workgroup g + 1 -- the next 4
//     sweeps, on any CU / XCD -- follows ~7 ticks behind.
// Workgroups are launched in group order (interleaved over the matrices of
// the batch), so a workgroup only waits on one that was dispatched before
// it; every wait is bounded (error count, then it proceeds) so a fault can
// never leave waves spinning.
// One task = one wave: the reflector on lanes 0-15, then the left block,
// the diagonal block and the block below side by side on lanes 0-15, 16-31,
// 32-47 in ONE instruction stream (16 LDS loads, 16 FMAs for the dot, two
// FMAs per element for the update, 16 LDS stores per lane).
//
// Outputs: d, e of the tridiagonal matrix (each finished as the sweep that
// touched it last leaves it), and the reflectors for the back-transformation
// (csrc/eig_q2.hip), one 16-float segment per task: v2[s][16 j] = tau,
// v2[s][16 j + i] = v[i] (v[0] = 1 implicit), zero past the reflector.
#include "common.h"

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <type_traits>
#include <vector>

namespace {

constexpr int SB = 16;            // half-bandwidth
constexpr int BW = 2 * SB;        // stored floats per band row
constexpr int RS = 36;            // LDS row stride (16-B aligned rows; conflict-free strides)
constexpr int NSLOT = 4;          // ring blocks per wave
constexpr int NW4 = 4;            // waves (sweeps) per workgroup (default; 8 with KFAC_SB2ST_DBG & 32)
constexpr int LAG = 3;            // ticks between consecutive sweeps
constexpr int SLOTF = SB * RS;    // floats per ring block
constexpr int SC1 = 16;           // buffer-op cache policy: sc1 (write-through / L1-bypass)
constexpr int DONE = 1 << 30;     // published count of a finished sweep
constexpr int SPIN_MAX = 1 << 22; // bounded waits (~0.3 s)
constexpr int MAXMAT = 64;

struct SbMat {
  float* band;            // (n + 32) x 32 band from stage 1, reduced in place
  float* v2;              // (n - 1) x ldv2 reflectors, zeroed by the caller
  float* d;
  float* e;
  int* prog;              // [groups] published block count of each group's last sweep
  int* err;               // bounded waits that timed out (0 when healthy)
  long long ldv2;
  int n, dbg;             // dbg (timing experiments, KFAC_SB2ST_DBG): 1 = no polls, 2 = no publish wait,
                          // 8 = per-workgroup start / end stamps, 16 = XCD-affine workgroup order
  long long* ts;          // dbg & 8: [workgroup][2] s_memrealtime stamps (100 MHz); dbg & 128:
                          // then 8 ticks x 8 phase stamps (s_memtime) of group 0's wave 1
  int nwg;                // workgroups of the launch (stamp layout)
  int* status;            // caller's int: the timed-out wait count after the launch (host check)
};
struct SbWg { int mat, g; };

__device__ __forceinline__ int sweep_tasks(int n, int s) {
  // tasks j with r0 = s + 1 + 16 j <= n - 2 (a reflector of length >= 2)
  return (s + 1 <= n - 2) ? (n - 3 - s) / SB + 1 : 0;
}

// 16-lane row sum (DPP inside each row of 16 lanes; every lane gets its row's sum)
__device__ __forceinline__ float row_sum16(float v) {
  v += dpp_f<0xB1>(v);     // quad_perm [1,0,3,2]
  v += dpp_f<0x4E>(v);     // quad_perm [2,3,0,1]
  v += dpp_f<0x141>(v);    // row_half_mirror
  v += dpp_f<0x140>(v);    // row_mirror
  return v;
}

__device__ __forceinline__ float rdlane(float v, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}

// value of lane (lane & 15) of row 0 for every lane (v lives on lanes 0..15)
__device__ __forceinline__ float rdlane_row(float v, int li) {
  return __shfl(v, li, 64);
}

__device__ __forceinline__ fx4 band_ld(__amdgpu_buffer_rsrc_t rs, int byte_off) {
  return __builtin_amdgcn_raw_buffer_load_b128(rs, byte_off, 0, SC1);
}

// spin (bounded) until *p >= need; sc1 polls
// (after one timeout anywhere every later wait returns at once: a broken
// pipeline ends in ~one SPIN_MAX, with garbage results and err > 0)
__device__ __forceinline__ void wait_count(int* p, int need, int* err) {
  if (need <= 0) return;
  int it = 0;
  while (__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < need) {
    __builtin_amdgcn_s_sleep(1);
    if ((++it & 1023) == 0 &&
        __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0)
      break;
    if (it == SPIN_MAX) {
      atomicAdd(err, 1);
      break;
    }
  }
}

// LDS layout of a workgroup (floats): the NW compute waves' rings, the IO
// wave's staging ring for wave 0, the poll words, one dummy word per wave
constexpr int NST = 8;            // staging slots (16 rows x 32 floats, lane-linear DMA image)
constexpr int STF = SB * BW;      // floats per staging slot
constexpr int PD = 4;             // IO wave: blocks loaded PD ticks ahead of wave 0's use
template <int NW> constexpr int lds_floats() { return NW * NSLOT * SLOTF + NST * STF + 4 * 64 + NW + 1; }

// LDS-DMA (buffer_load ... lds): each lane's `size` bytes land at base + lane * size
__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t rs, float* lds_base, int voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)lds_base, 16,
                                           voff, 0, 0, SC1);
}
__device__ __forceinline__ void dma4(__amdgpu_buffer_rsrc_t rs, int* lds_base, int voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)lds_base, 4,
                                           voff, 0, 0, SC1);
}

// Waves 0 .. NW-1 run the sweeps (as before); wave NW is the IO wave: it
// polls the predecessor group's published count and streams wave 0's band
// blocks into LDS with LDS-DMA, PD ticks ahead, with COUNTED waits only (no
// VGPR destinations, so no compiler-inserted vmcnt(0)): its tick issues
// exactly three memory ops -- the poll DMA for tick t + 2 and the two 1-KB
// DMAs of block t + PD -- and first waits vmcnt(3), i.e. for everything of
// ticks <= t - 2 (block t + 2, wave 0's next copy, and the poll it reads now).
// Round 3's register prefetch in wave 0 waited vmcnt(0) after every load
// (register copies at the set merge) and its poll drained the queue: a
// global round trip inside every other tick.
template <int NW>
__global__ __launch_bounds__(64 * (NW + 1)) void sb2st_kernel(const SbMat* __restrict__ mats,
                                                             const SbWg* __restrict__ wgs) {
  const SbWg W = wgs[blockIdx.x];
  if (W.mat < 0) return;                         // XCD-affine order: padding slot
  const SbMat M = mats[W.mat];
  if (M.ts && threadIdx.x == 0) M.ts[2 * blockIdx.x] = (long long)__builtin_amdgcn_s_memrealtime();
  const int n = M.n, grp = W.g;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  extern __shared__ float lds[];
  float* stage = lds + NW * NSLOT * SLOTF;       // NST slots
  int* polls = (int*)(stage + NST * STF);        // 4 x 64 words
  float* dummy = (float*)(polls + 4 * 64) + w;   // one spare word per wave
  float* my = lds + (w < NW ? w : 0) * (NSLOT * SLOTF);
  const float* prod = lds + ((w + NW - 1) % NW) * (NSLOT * SLOTF);
  AS1 float* v2 = gptr(M.v2);
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      M.band, 0, (n + BW) * BW * 4, 0x00020000);
  if (grp == 0 && tid == 0) {
    const fx4 r0 = band_ld(rs, 28 * 4);
    M.d[0] = r0.w;
    if (n == 2) {
      const fx4 r1 = band_ld(rs, (BW + 28) * 4);
      M.d[1] = r1.w; M.e[0] = r1.z;
    }
  }
  const int nsw = n - 2;                          // sweeps with tasks: 0 .. n - 3
  const int s0 = grp * NW;                        // wave 0's sweep
  const int s = s0 + (w < NW ? w : 0);
  const int J = (w < NW && s < nsw) ? sweep_tasks(n, s) : 0;
  const int J0 = s0 < nsw ? sweep_tasks(n, s0) : 0;
  int T = 0;                                      // ticks of the group (uniform)
#pragma unroll 1
  for (int ww = 0; ww < NW; ++ww) {
    const int ss = s0 + ww;
    const int jj = ss < nsw ? sweep_tasks(n, ss) : 0;
    if (jj > 0) T = max(T, LAG * ww + jj);
  }
  // copy lane: block row i = lane >> 2, quarter qd = lane & 3 (8 floats)
  const int ci = lane >> 2, cq = lane & 3;
  const int g = lane >> 4, li = lane & 15;
  int* prev = grp > 0 ? M.prog + grp - 1 : nullptr;
  int* mine = M.prog + grp;
  const bool polling = prev && !(M.dbg & 1);
  // producer blocks (previous group's last sweep s0 - 1) that block k of
  // wave 0's sweep needs: rows s0+1+16k .. min(s0+16+16k, n-1)
  // (a block past the band's end still needs every producer block up to the
  // last row: returning 0 there let the prologue, which asks for block PD-1,
  // skip the wait on small matrices and read stale rows)
  auto need_of = [&](int k) {
    const int rhi = min(s0 + SB + SB * k, n - 1);
    if (rhi < s0 + 1) return 0;
    return (rhi - s0) / SB + 1;
  };
  // IO wave: block k of wave 0's sweep (rows s0+1+16k ..: 2 KB contiguous in
  // the band; rows n .. n+31 are zero, rows past them out of range -> zero)
  auto dma_block = [&](int k) {
    float* dst = stage + (k % NST) * STF;
    const int vo = (s0 + 1 + SB * k) * BW * 4 + lane * 16;
    dma16(rs, dst, vo);
    dma16(rs, dst + 256, vo + 1024);
  };
  const __amdgpu_buffer_rsrc_t rsp = __builtin_amdgcn_make_buffer_rsrc(
      M.prog, 0, (grp + 1) * 4, 0x00020000);
  const int poll_off = (grp > 0 ? grp - 1 : grp) * 4;
  if (w == NW) {
    if (J0 > 0) {
      int c0 = 0;
      if (polling) {
        wait_count(prev, need_of(PD - 1), M.err);
        c0 = __hip_atomic_load(prev, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      for (int k = 0; k < PD; ++k) dma_block(k);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (lane == 0) { polls[2 * 64] = c0; polls[3 * 64] = c0; }
    }
  }
  kfac_lds_barrier();
  // wave 0 copies block k from the staging slot (rows of 32) into its ring
  auto lput = [&](int k) {
    const float* src = stage + (k % NST) * STF + ci * BW + cq * 8;
    float* dst = my + (k % NSLOT) * SLOTF + ci * RS + cq * 8;
    *(fx4*)dst = *(const fx4*)src;
    *(fx4*)(dst + 4) = *(const fx4*)(src + 4);
  };
  if (w == 0 && J > 0) lput(0);
  // fill my block k from the previous wave's blocks k (rows 1..15) and
  // k + 1 (row 0); rows past n read as zero
  auto ring_fill = [&](int k) {
    const int r = s + 1 + SB * k + ci;
    const float* src = (ci < SB - 1) ? prod + (k % NSLOT) * SLOTF + (ci + 1) * RS
                                     : prod + ((k + 1) % NSLOT) * SLOTF;
    fx4 a = *(const fx4*)(src + cq * 8);
    fx4 b = *(const fx4*)(src + cq * 8 + 4);
    const fx4 z = {0.f, 0.f, 0.f, 0.f};
    float* dst = my + (k % NSLOT) * SLOTF + ci * RS + cq * 8;
    *(fx4*)dst = r < n ? a : z;
    *(fx4*)(dst + 4) = r < n ? b : z;
  };
  auto band_st = [&](int k) {
    const int r = s + 1 + SB * k + ci;
    const float* src = my + (k % NSLOT) * SLOTF + ci * RS + cq * 8;
    if (r < n) {
      __builtin_amdgcn_raw_buffer_store_b128(*(const fx4*)src, rs, (r * BW + cq * 8) * 4, 0, SC1);
      __builtin_amdgcn_raw_buffer_store_b128(*(const fx4*)(src + 4), rs, (r * BW + cq * 8 + 4) * 4,
                                             0, SC1);
    }
  };

#pragma unroll 1
  for (int t = 0; t < T; ++t) {
    if (w == NW) {
      // ---- IO wave: ticks <= t - 2 landed (block t + 2, the poll of t - 2)
      asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
      if (t + PD < J0 + 2) {
        if (polling) {
          const int c = polls[((t + 2) & 3) * 64];
          const int need = need_of(t + PD);
          if (c < need) wait_count(prev, need, M.err);   // slow path (drains the queue)
        }
      }
      dma4(rsp, polls + (t & 3) * 64, poll_off);
      dma_block(t + PD);
      kfac_lds_barrier();
      continue;
    }
    const int j = t - LAG * w;
#ifdef SB2ST_PHASE_STAMPS
    // (compile-time only: the stamps' SMEM / flat ops share lgkmcnt with the
    // LDS reads and make every LDS wait a full drain)
    const bool stamp = (M.dbg & 128) && M.ts && grp == 0 && w == 1 && t >= 20 && t < 28;
#define SB2ST_IF if (stamp)
#else
    constexpr bool stamp = false;
#define SB2ST_IF if constexpr (false)
#endif
    long long* st = stamp ? M.ts + 2 * M.nwg + (t - 20) * 8 : nullptr;
#define SB2ST_STAMP(ph)                                                     \
    SB2ST_IF { if (lane == 0) st[ph] = (long long)__builtin_amdgcn_s_memtime(); }
    SB2ST_STAMP(0)
    if (w > 0 && J > 0 && j == -1) ring_fill(0);
    if (j >= 0 && j < J) {
      // ---- block j + 1 (the rows below this task's reflector)
      if (w == 0) lput(j + 1);
      else ring_fill(j + 1);
      SB2ST_STAMP(1)
      if (w == NW - 1) {
        // publish the blocks stored two tasks ago: this wave's vector memory
        // ops per task are the V2 store then the two band stores, so with
        // the previous task's three still in flight (vmcnt(3)) every older
        // band store has completed
        if (!(M.dbg & 2)) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
        __hip_atomic_store(mine, j > 0 ? j - 1 : 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      const int r0 = s + 1 + SB * j;
      const int L = min(SB, n - r0);            // >= 2
      float* S0 = my + (j % NSLOT) * SLOTF;
      float* S1 = my + ((j + 1) % NSLOT) * SLOTF;
      // ---- every LDS operand of the task first (none depends on the
      // reflector): element l of this lane's vector, branch-free
      //   g0 (left, j >= 1): column c+1+li, row l     -> S0 + 16 + li + 35 l
      //   g1 (diagonal, row li): l <= li -> S0 + 35 li + 31 + l
      //                          l >  li -> S0 + 35 l + li + 31
      //   g2 (below, row 16+li): column r0+l           -> S1 + 35 li + 15 + l
      // inactive lanes (g0 at j = 0 or li = 15, g3) read and write a dummy word
      const bool g0 = g == 0, g1 = g == 1, g2 = g == 2;
      const bool act = (g0 && j > 0 && li < SB - 1) || g1 || g2;
      float* P = g2 ? S1 : S0;
      const int boff = g0 ? 16 + li : (g1 ? 35 * li + 31 : 35 * li + 15);
      const int bstr = g0 ? 35 : 1;
      float* addr[SB];
#pragma unroll
      for (int l = 0; l < SB; ++l) {
        const int off = (g1 && l > li) ? 35 * l + li + 31 : boff + bstr * l;
        addr[l] = act ? P + off : dummy;
      }
      // ---- reflector column c first (lanes 0..15: row i = lane): the
      // reflector math then runs while the 16 operand reads are in flight
      const int xo = (j == 0) ? 30 : 15;        // column c's offset in row i: xo - i
      float* xp = S0 + 35 * (lane & 15) + xo;
      // (asm read + counted wait: the compiler's own wait for a value read
      // before the 16 operand reads is lgkmcnt(0), i.e. all 17)
      float xl;
      asm volatile("ds_read_b32 %0, %1" : "=v"(xl) : "v"((unsigned)(size_t)xp) : "memory");
      float val[SB];
#pragma unroll
      for (int l = 0; l < SB; ++l) val[l] = *addr[l];
      asm volatile("s_waitcnt lgkmcnt(15)" : "+v"(xl) :: "memory");   // (4-bit field: x and the first operand)
      const float x = (lane < L) ? xl : 0.f;
      SB2ST_IF { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
      SB2ST_STAMP(2)
      const float alpha = rdlane(x, 0);
      // x lives on lanes 0..15: a 16-lane (DPP row) sum, read from lane 0
      const float sig = rdlane(row_sum16((lane >= 1 && lane < L) ? x * x : 0.f), 0);
      float tau = 0.f, beta = alpha, scal = 0.f;
      if (sig != 0.f) {
        beta = -copysignf(__builtin_sqrtf(alpha * alpha + sig), alpha);
        tau = (beta - alpha) * __builtin_amdgcn_rcpf(beta);
        scal = __builtin_amdgcn_rcpf(alpha - beta);
      }
      const float v = lane == 0 ? 1.f : ((lane < L) ? x * scal : 0.f);
      SB2ST_STAMP(3)
      if (lane < L) {
        *xp = lane == 0 ? beta : 0.f;
        v2[(long long)s * M.ldv2 + SB * j + lane] = lane == 0 ? tau : v;
      }
      if (tau != 0.f) {
        float vl[SB];
#pragma unroll
        for (int l = 0; l < SB; ++l) vl[l] = rdlane(v, l);
        float d0 = 0.f, d1 = 0.f, d2 = 0.f, d3 = 0.f;
#pragma unroll
        for (int l = 0; l < SB; l += 4) {
          d0 += val[l] * vl[l]; d1 += val[l + 1] * vl[l + 1];
          d2 += val[l + 2] * vl[l + 2]; d3 += val[l + 3] * vl[l + 3];
        }
        const float dot = (d0 + d1) + (d2 + d3);
        // g1: w = tau D v - K v, K = tau / 2 v^T (tau D v)
        // (the exchange outside the select: a ?: arm is divergent code)
        const float vsh = __shfl_xor(v, 16, 64);   // lane 16 + li <- lane li (v_permlane16_swap)
        const float vli = g1 ? vsh : 0.f;
        const float p = tau * dot;
        const float kk = 0.5f * tau * row_sum16(vli * p);
        const float wv = p - kk * vli;
        SB2ST_STAMP(4)
        float wl[SB];
#pragma unroll
        for (int l = 0; l < SB; ++l) wl[l] = rdlane(wv, 16 + l);
        // update: g0 / g2 -= (tau dot) v[l]; g1 -= w v[l] + v[li] w[l] (lower only)
        const float a1 = g1 ? wv : p;
        const float a2 = g1 ? vli : 0.f;
#pragma unroll
        for (int l = 0; l < SB; ++l) {
          const float nv = val[l] - (a1 * vl[l] + a2 * wl[l]);
          float* pa = (g1 && l > li) ? dummy : addr[l];
          *pa = nv;
        }
      }
      SB2ST_STAMP(5)
      // ---- outputs finished by this task
      if (j == 0 && lane == 0) {
        M.d[s + 1] = S0[31];
        M.e[s] = S0[30];
        if (s == n - 3) { M.d[n - 1] = S0[RS + 31]; M.e[n - 2] = S0[RS + 30]; }
      }
      // ---- the group's last sweep hands its finished blocks to the next group
      if (w == NW - 1) {
        band_st(j);
        if (j == J - 1) {
          band_st(j + 1);
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          __hip_atomic_store(mine, DONE, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      }
    }
    SB2ST_IF { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
    SB2ST_STAMP(6)
    kfac_lds_barrier();
    SB2ST_STAMP(7)
#undef SB2ST_STAMP
#undef SB2ST_IF
  }
  if (w == NW) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // no DMA outlives the group
  // a group whose last sweep has no task still releases its successor
  if (w == NW - 1 && J == 0 && lane == 0)
    __hip_atomic_store(mine, DONE, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (M.ts && threadIdx.x == 0) M.ts[2 * blockIdx.x + 1] = (long long)__builtin_amdgcn_s_memrealtime();
}

__global__ __launch_bounds__(256) void sb2st_zero_kernel(int* p, int n) {
  for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) p[i] = 0;
}

struct SbPlan {
  SbMat* d_mats = nullptr;
  SbWg* d_wgs = nullptr;
  int* d_prog = nullptr;       // all matrices' group counters, then the error count
  int nprog = 0, nwg = 0, nw = NW4, count = 0;
  long long* d_ts = nullptr;
  hipGraphExec_t exec = nullptr;
};

long long* g_last_ts = nullptr;
int g_last_nwg = 0;
std::vector<SbWg> g_last_wgs;

// 37 KB of ring per workgroup, padded so that exactly one workgroup sits on a
// CU (the sc1 hand-off's measured form)
constexpr size_t LDS_BYTES = 96 * 1024;
static_assert((size_t)lds_floats<8>() * sizeof(float) <= LDS_BYTES, "ring exceeds LDS");

// after the pipeline: every matrix's status word = the launch's timed-out wait
// count (a broken pipeline finishes with garbage d / e / v2; the host raises
// on a nonzero status in eigen.check_solver_status)
__global__ void sb2st_status_kernel(const SbMat* __restrict__ mats, int count) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < count && mats[i].status != nullptr)
    *mats[i].status = __hip_atomic_load(mats[i].err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

int enqueue(const SbPlan& P, hipStream_t s) {
  hipLaunchKernelGGL(sb2st_zero_kernel, dim3(4), dim3(256), 0, s, P.d_prog, P.nprog + 1);
  if (P.nw == 8)
    hipLaunchKernelGGL(sb2st_kernel<8>, dim3(P.nwg), dim3(64 * 9), LDS_BYTES, s, P.d_mats, P.d_wgs);
  else
    hipLaunchKernelGGL(sb2st_kernel<NW4>, dim3(P.nwg), dim3(64 * (NW4 + 1)), LDS_BYTES, s,
                       P.d_mats, P.d_wgs);
  hipLaunchKernelGGL(sb2st_status_kernel, dim3((P.count + 63) / 64), dim3(64), 0, s, P.d_mats,
                     P.count);
  return (int)hipGetLastError();
}

std::mutex g_mu;
std::map<std::string, SbPlan> g_plans;

}  // namespace

// dbg & 8: copy the last plan's stamps out: per workgroup (mat, group, start, end)
KFAC_API int kfac_sb2st_debug_stamps(long long* out, int max_wg) {
  if (!g_last_ts) return 0;
  const int nw = std::min(max_wg, g_last_nwg);
  std::vector<long long> t(2 * (size_t)g_last_nwg);  // (the phase stamps follow)
  if (hipMemcpy(t.data(), g_last_ts, sizeof(long long) * t.size(), hipMemcpyDeviceToHost) != hipSuccess)
    return -1;
  for (int b = 0; b < nw; ++b) {
    out[4 * b] = g_last_wgs[b].mat; out[4 * b + 1] = g_last_wgs[b].g;
    out[4 * b + 2] = t[2 * b]; out[4 * b + 3] = t[2 * b + 1];
  }
  return nw;
}

// dbg & 128: the 64 phase stamps (8 ticks x 8 phases, s_memtime cycles)
KFAC_API int kfac_sb2st_debug_phases(long long* out) {
  if (!g_last_ts) return 0;
  return (int)hipMemcpy(out, g_last_ts + 2 * g_last_nwg, sizeof(long long) * 64,
                        hipMemcpyDeviceToHost);
}

struct KfacSb2stRecord {
  const float* band_in; float* band; float* v2; float* d; float* e; long long ldv2; long long n;
  int* status;   // nullptr, or an int that receives the timed-out wait count
};

// Band -> tridiagonal for `count` matrices (n >= 2): band ((n+32) x 32, the
// stage-1 lower band, reduced in place; band_in must equal band), v2 ((n-1) x
// ldv2, ldv2 >= n + 16, zeroed by the caller), d (n), e (n-1).  A pipeline of
// ceil((n-2)/4) workgroups per matrix.
KFAC_API int kfac_sb2st_batched(const KfacSb2stRecord* recs, int count, int use_graph,
                                hipStream_t stream) {
  if (count > MAXMAT) return -5;
  if (count <= 0) return 0;
  static bool attr = false;
  if (!attr) {
    if (hipFuncSetAttribute((const void*)sb2st_kernel<NW4>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)LDS_BYTES) != hipSuccess ||
        hipFuncSetAttribute((const void*)sb2st_kernel<8>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)LDS_BYTES) != hipSuccess)
      return -7;
    attr = true;
  }
  std::vector<SbMat> mats(count);
  std::vector<int> ngrp(count);
  int nprog = 0;
  for (int i = 0; i < count; ++i) {
    const KfacSb2stRecord& r = recs[i];
    if (r.n < 2 || r.ldv2 < r.n + SB || r.band_in != r.band) return -2;
    SbMat& M = mats[i];
    memset(&M, 0, sizeof(M));
    M.band = r.band; M.v2 = r.v2; M.d = r.d; M.e = r.e;
    M.ldv2 = r.ldv2; M.n = (int)r.n; M.status = r.status;
    M.dbg = getenv("KFAC_SB2ST_DBG") ? atoi(getenv("KFAC_SB2ST_DBG")) : 0;
    const int nsw = (int)r.n - 2;
    const int nw = (M.dbg & 32) ? 8 : NW4;
    ngrp[i] = nsw > 0 ? (nsw + nw - 1) / nw : 1;
    nprog += ngrp[i];
  }
  hipStreamCaptureStatus cst = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(stream, &cst) != hipSuccess) return -3;
  const bool graph = use_graph && stream != nullptr && cst == hipStreamCaptureStatusNone;
  const std::string key((const char*)mats.data(), sizeof(SbMat) * mats.size());
  SbPlan* plan;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    auto it = g_plans.find(key);
    if (it == g_plans.end()) {
      SbPlan P;
      P.nw = (mats[0].dbg & 32) ? 8 : NW4;
      P.count = count;
      int err;
      if ((err = (int)hipMalloc(&P.d_prog, sizeof(int) * (nprog + 1))) != 0) return err;
      P.nprog = nprog;
      int off = 0;
      for (int i = 0; i < count; ++i) {
        mats[i].prog = P.d_prog + off;
        mats[i].err = P.d_prog + nprog;
        off += ngrp[i];
      }
      // launch order: group-major, interleaved over matrices, so every
      // workgroup's predecessor (same matrix, group - 1) was dispatched first
      std::vector<SbWg> wgs;
      int gmax = 0;
      for (int i = 0; i < count; ++i) gmax = std::max(gmax, ngrp[i]);
      const int dbg = mats[0].dbg;
      if ((dbg & 16) && count <= 8) {
        // workgroup b runs on XCD b mod 8 (round-robin dispatch): matrix i's
        // groups all on XCD i, padding slots exit at once
        for (int g = 0; g < gmax; ++g)
          for (int x = 0; x < 8; ++x)
            wgs.push_back(x < count && g < ngrp[x] ? SbWg{x, g} : SbWg{-1, 0});
      } else {
        for (int g = 0; g < gmax; ++g)
          for (int i = 0; i < count; ++i)
            if (g < ngrp[i]) wgs.push_back(SbWg{i, g});
      }
      P.nwg = (int)wgs.size();
      if (dbg & 8) {
        if ((err = (int)hipMalloc(&P.d_ts, sizeof(long long) * (2 * P.nwg + 64))) != 0) return err;
        for (auto& M : mats) { M.ts = P.d_ts; M.nwg = P.nwg; }
        g_last_ts = P.d_ts; g_last_nwg = P.nwg; g_last_wgs = wgs;
      }
      if ((err = (int)hipMalloc(&P.d_mats, sizeof(SbMat) * count)) != 0) return err;
      if ((err = (int)hipMemcpy(P.d_mats, mats.data(), sizeof(SbMat) * count,
                                hipMemcpyHostToDevice)) != 0)
        return err;
      if ((err = (int)hipMalloc(&P.d_wgs, sizeof(SbWg) * wgs.size())) != 0) return err;
      if ((err = (int)hipMemcpy(P.d_wgs, wgs.data(), sizeof(SbWg) * wgs.size(),
                                hipMemcpyHostToDevice)) != 0)
        return err;
      it = g_plans.emplace(key, P).first;
    }
    plan = &it->second;
    if (graph && !plan->exec) {
      static hipStream_t cap = nullptr;
      if (!cap && hipStreamCreateWithFlags(&cap, hipStreamNonBlocking) != hipSuccess) cap = nullptr;
      hipGraph_t gr = nullptr;
      if (cap && hipStreamBeginCapture(cap, hipStreamCaptureModeThreadLocal) == hipSuccess) {
        const int e1 = enqueue(*plan, cap);
        const hipError_t e2 = hipStreamEndCapture(cap, &gr);
        if (!e1 && e2 == hipSuccess && gr &&
            hipGraphInstantiate(&plan->exec, gr, nullptr, nullptr, 0) != hipSuccess)
          plan->exec = nullptr;
        if (gr) (void)hipGraphDestroy(gr);
      }
      (void)hipGetLastError();
    }
  }
  if (graph && plan->exec) return (int)hipGraphLaunch(plan->exec, stream);
  return enqueue(*plan, stream);
}
