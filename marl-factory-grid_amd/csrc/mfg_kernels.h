// mfg_kernels.h — device code of the MI355X batched step engine (all kernels and their device functions).
// Included by mfg_engine.hip (host side, C-ABI, every kernel but the observation render) and by the
// mfg_obs_*.hip translation units, each of which instantiates the observation-render kernels for a subset of
// ray lengths (launch_obs_inst): the render has ~240 instantiations and the split lets them compile in parallel.
#pragma once
//
// Replaces, for a batch of B independent environments:
//   Factory.reset / Factory.step       marl_factory_grid/environment/factory.py:134-148, 189-259
//   Gamestate.tick / check_done        marl_factory_grid/utils/states.py:170-226
//   rule hooks + actions of the modules listed in mfg.h
//   OBSBuilder.build_for_all           marl_factory_grid/utils/observation_builder.py:96-235
// bit-exactly, including the reference's RNG streams (CPython MT19937 floor shuffles, numpy PCG64
// uniform draws) and its documented quirks.
//
// See mfg_device.h for the execution model (one wavefront per env).
#include <hip/hip_runtime.h>
// Build switches are compile-time only (-D...); nothing is read from the environment at run time (the parity
// tests force exact alternative paths through the test-only mfg_create_variant, include/mfg.h):
//   MFG_RESET_OVERLAP      resets + their renders on a second stream beside the render (below)
//   MFG_REPLAY2            the two-wave replay: 1 by occupancy (default), 2 always (the parity suite runs it on C2-C4)
#ifndef MFG_RESET_OVERLAP
// mfg_step with auto-reset: the resets + their renders on a second stream beside the other envs' render.
// 0 never, 1 when the reset is long (agents x floor cells >= 16384: the per-agent floor shuffles and draws of
// SpawnAgents, C4/C5), 2 always
#define MFG_RESET_OVERLAP 1
#endif
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>
#include <vector>
#include <algorithm>
#include <type_traits>

#include "mfg_device.h"

typedef unsigned long long u64;

// ------------------------------------------------------------------------------------------------
// wave primitives
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ int lane_id() { return (int)__lane_id(); }
__device__ __forceinline__ u64 ballot(bool p) { return (u64)__ballot(p); }
__device__ __forceinline__ int popc(u64 m) { return __popcll(m); }
__device__ __forceinline__ u64 lt_mask() { return (1ull << lane_id()) - 1ull; }
// mbcnt(m) in two VALU ops
__device__ __forceinline__ int mbcnt(u64 m) {
  return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}
// a wave mask (SGPR pair) as a per-lane predicate, free (the mask is used as the condition directly)
__device__ __forceinline__ bool lanes(u64 m) { return __builtin_amdgcn_inverse_ballot_w64(m); }
__device__ __forceinline__ int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ int ffs64(u64 m) { return __ffsll((long long)m) - 1; }
__device__ __forceinline__ int rl(int v, int l) { return __builtin_amdgcn_readlane(v, l); }
__device__ __forceinline__ double rld(double v, int l) {
  const unsigned long long b = __double_as_longlong(v);
  const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)b, l);
  const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(b >> 32), l);
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}
__device__ __forceinline__ u64 wave_or64(u64 v) {
  unsigned lo = (unsigned)v, hi = (unsigned)(v >> 32);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    lo |= __shfl_xor(lo, o);
    hi |= __shfl_xor(hi, o);
  }
  return ((u64)hi << 32) | lo;
}

// ------------------------------------------------------------------------------------------------
// per-wave env context: the env record is mirrored 1:1 in the wave's LDS slice
// ------------------------------------------------------------------------------------------------
// The spec is read through the constant address space: uniform loads from it become scalar loads.
#define CS __attribute__((address_space(4)))
typedef const CS MfgDevSpec* SpecP;

struct Env {
  SpecP S;
  uint8_t* lds;     // this wave's LDS slice == image of the HBM record
  int* scratch;     // 512 ints after the record (spawn positions, id-collision pairs)
  uint32_t* stab;   // [MFG_STAB_N] tagged max-tables of the parallel shuffle blocks (not persisted)
  uint8_t* cmap;    // [HW] per-env cell map of the obs render (u8 cells, u16 with machines/maintainers)
  uint8_t* bfs;     // maintainer BFS scratch (full-record kernels of specs with MoveMaintainers)
  int* hdrp;        // header slots (inside the record image, or a separate slice in k_replay)
  int lane;
  int mdelta = 0;   // where the maintainer states sit relative to their record offset (k_logic<.., SEL 1>)
  const uint16_t* gpath = nullptr;  // k_logic<.., SEL 1>: the maintainer paths read in place in the HBM record
  __device__ int* hdr() const { return hdrp; }
  __device__ int* rctr() const { return (int*)(lds + S->L.o_rule_ctr); }
  __device__ int* agpos() const { return (int*)(lds + S->L.o_agent_pos); }
  __device__ int* agarr() const { return (int*)(lds + S->L.o_agent_arr); }
  __device__ int* agpar() const { return (int*)(lds + S->L.o_agent_par); }
  __device__ int* forg() const { return (int*)(lds + S->L.o_frozen_org); }
  __device__ int* fgp() const { return (int*)(lds + S->L.o_frozen_gp); }
  __device__ int* door() const { return (int*)(lds + S->L.o_door); }
  __device__ int* items() const { return (int*)(lds + S->L.o_items); }
  __device__ int* pods() const { return (int*)(lds + S->L.o_pods); }
  __device__ int* drops() const { return (int*)(lds + S->L.o_drops); }
  __device__ int* dests() const { return (int*)(lds + S->L.o_dests); }
  __device__ int* dirtpos() const { return (int*)(lds + S->L.o_dirt_pos); }
  __device__ int* dirtid() const { return (int*)(lds + S->L.o_dirt_id); }
  __device__ double* bat() const { return (double*)(lds + S->L.o_battery); }
  __device__ double* fbat() const { return (double*)(lds + S->L.o_frozen_bat); }
  __device__ double* dirtamt() const { return (double*)(lds + S->L.o_dirt_amt); }
  __device__ uint64_t* pcg() const { return (uint64_t*)(lds + S->L.o_pcg); }
  __device__ uint32_t* mt() const { return (uint32_t*)(lds + S->L.o_mt); }
  __device__ uint16_t* perm() const { return (uint16_t*)(lds + S->L.o_perm); }
  __device__ int* machines() const { return (int*)(lds + S->L.o_machines); }
  __device__ int* maints() const { return (int*)(lds + S->L.o_maints); }
  __device__ int* mst(int k) const { return (int*)(lds + S->L.o_mstate + mdelta) + k * S->mstate_ints; }
  __device__ uint16_t* mpath(int k) const { return (uint16_t*)(lds + S->L.o_mpath) + k * S->path_cap; }
  // a maintainer's path cell for reading (in place in HBM in k_logic<.., SEL 1>, else the record image)
  __device__ int mpath_at(int k, int i) const {
    return gpath ? (int)gpath[(size_t)k * S->path_cap + i] : (int)mpath(k)[i];
  }
  __device__ uint16_t* grank() const { return (uint16_t*)(lds + S->L.o_grank); }
  // uniform header access
  __device__ int H(int k) const { return uni(hdr()[k]); }
  __device__ void setH(int k, int v) const {
    if (lane == 0) hdr()[k] = v;
  }
};

__device__ __forceinline__ void wave_sync() { __builtin_amdgcn_wave_barrier(); __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront"); }
// lanes exchange through HBM scratch (BFS pool, pair spill): workgroup-scope fence (s_waitcnt on LDS and
// vector memory), then the wave barrier
__device__ __forceinline__ void mem_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
  __builtin_amdgcn_wave_barrier();
}

// ------------------------------------------------------------------------------------------------
// MT19937 (CPython semantics) — state in LDS, lane-parallel twist
// ------------------------------------------------------------------------------------------------
#define MT_UPPER 0x80000000u
#define MT_LOWER 0x7fffffffu
#define MT_MATRIX 0x9908b0dfu

// v_bitop3_b32 (gfx950): LUT 0x78 = a ^ (b & c), 0xE4 = c ? a : b bitwise (a = 0xF0, b = 0xCC, c = 0xAA)
#define XOR_AND(a, b, c) __builtin_amdgcn_bitop3_b32((a), (b), (c), 0x78)
__device__ __forceinline__ uint32_t mt_temper(uint32_t y) {
  y ^= (y >> 11);
  y = XOR_AND(y, y << 7, 0x9d2c5680u);
  y = XOR_AND(y, y << 15, 0xefc60000u);
  y ^= (y >> 18);
  return y;
}
__device__ __forceinline__ uint32_t mt_temper3(uint32_t y) {  // mt_temper without its last step
  y ^= (y >> 11);
  y = XOR_AND(y, y << 7, 0x9d2c5680u);
  return XOR_AND(y, y << 15, 0xefc60000u);
}
__device__ __forceinline__ uint32_t mt_mix(uint32_t a, uint32_t b, uint32_t c) {
  const uint32_t y = __builtin_amdgcn_bitop3_b32(a, b, MT_UPPER, 0xE4);  // (a & UPPER) | (b & LOWER)
  const uint32_t odd = (uint32_t)__builtin_amdgcn_sbfe((int)b, 0, 1);       // y & 1 == b & 1, as a mask
  return XOR_AND(c ^ (y >> 1), odd, MT_MATRIX);
}
// In-place twist in its three dependency phases (i<227: old inputs; 227<=i<454: mt[i-227] new;
// 454<=i<623: mt[i-227] new). Each phase issues all its LDS reads before any of its writes, so one
// wave pays three LDS round trips per 624 draws. (Taking mt[i+1] from the neighbour lane by DPP wave_shl
// instead of a third LDS read was bit-exact and measured no faster: k_replay 11.05-11.12 vs 10.97-11.03 ms.)
// The third operand of phases 2 and 3, mt[i - 227], is the previous phase's result in the same lane and slot
// (i - 227 = i0 - 227 + t * 64 + lane), and new[623] takes old[623], new[0] and new[396] from lanes too. So no read
// waits on a write: the 26 reads of old words are issued first, then the writes, one sync per twist (was 33
// reads, 3 round trips and 4 syncs). Every address is one lane base plus an immediate offset: reads past a phase's
// end fetch words of the same slice (later MT words or the permutation) whose results are dropped, and only the
// last slot of each phase masks its writes, so no per-slot clamp or sink select runs on the VALU.
__device__ void mt_twist(const Env& e) {
  uint32_t* const p = e.mt() + e.lane;
  const int lane = e.lane;
  uint32_t a1[4], b1[4], c1[4], a2[4], b2[4], a3[3], b3[3];
#pragma unroll
  for (int t = 0; t < 4; t++) {
    a1[t] = p[t * MFG_WAVE]; b1[t] = p[t * MFG_WAVE + 1]; c1[t] = p[t * MFG_WAVE + 397];
  }
#pragma unroll
  for (int t = 0; t < 4; t++) {
    a2[t] = p[227 + t * MFG_WAVE]; b2[t] = p[227 + t * MFG_WAVE + 1];
  }
#pragma unroll
  for (int t = 0; t < 3; t++) {
    a3[t] = p[454 + t * MFG_WAVE]; b3[t] = p[454 + t * MFG_WAVE + 1];
  }
  uint32_t v1[4], v2[4], v3[3];
#pragma unroll
  for (int t = 0; t < 4; t++) v1[t] = mt_mix(a1[t], b1[t], c1[t]);
#pragma unroll
  for (int t = 0; t < 4; t++) v2[t] = mt_mix(a2[t], b2[t], v1[t]);
#pragma unroll
  for (int t = 0; t < 3; t++) v3[t] = mt_mix(a3[t], b3[t], v2[t]);
  // new[623] = mix(old[623], new[0], new[396]): old[623] is b3[2] of lane 40 (word 622 + 1), new[0] v1[0] of lane 0,
  // new[396] v2[2] of lane 41 (396 = 227 + 128 + 41)
  const uint32_t last = mt_mix((uint32_t)rl((int)b3[2], 40), (uint32_t)rl((int)v1[0], 0), (uint32_t)rl((int)v2[2], 41));
  // every read before any write: per lane the read and write offsets differ, so without a fence the compiler may
  // move a write above a read of another lane's word (e.g. lane 0's store of word 64 above lane 63's read of it)
  wave_sync();
#pragma unroll
  for (int t = 0; t < 3; t++) p[t * MFG_WAVE] = v1[t];  // words 0..191
#pragma unroll
  for (int t = 0; t < 3; t++) p[227 + t * MFG_WAVE] = v2[t];  // 227..418
#pragma unroll
  for (int t = 0; t < 2; t++) p[454 + t * MFG_WAVE] = v3[t];  // 454..581
  if (lane < 35) {  // 192..226 and 419..453
    p[3 * MFG_WAVE] = v1[3];
    p[227 + 3 * MFG_WAVE] = v2[3];
  }
  if (lane < 41) p[454 + 2 * MFG_WAVE] = v3[2];  // 582..622
  if (lane == 0) p[623] = last;
  wave_sync();
}

// Draw random.randbelow(i+1) for i = hi, hi-1, ..., lo (the inner loop of random.shuffle,
// random.py:380-395 with _randbelow_with_getrandbits, random.py:239-249). 64 draws are tempered in
// parallel; which draws are accepted (and for which i) is the fixed point of
//   A_l = #accepted lanes < l,  i_l = icur - A_l,  accept_l = (y_l >> (32 - bitlen(i_l+1))) <= i_l,
// found by Jacobi iteration with ballots (lane 0 is exact after 1 round, lane l after l+1; typical 2-3).
//
// If perm != null the accepted draws' Fisher-Yates swaps (i_t, j_t), t = accepted-lane order, are
// applied as ONE parallel block instead of a serial chain. Accepted ranks t have i_t = icur - t and
// j_t <= i_t, so:
//   V_t (value leaving i_t) = V_{pi(t)} if pi(t) = last s<t with j_s == i_t exists, else P0[i_t]
//   F_t (value landing on i_t) = V_{pj(t)} if pj(t) = last s<t with j_s == j_t exists, else P0[j_t]
// (P0 = block-start values). pi comes from a 64-entry tagged max-table keyed by rank (icur - j_s,
// self-swaps excluded); V by pointer jumping.
//  * exchange path (32-bit perm, S->xchg_ordered): one ds_wrxchg of V_t into perm[j_t] per lane. The
//    LDS applies a wave's conflicting lanes in ascending lane order (verified on the device by
//    mfg_create's probe, else this path is off), so lane t gets F_t back and the last writer stays.
//    Then perm[i_t] = F_t.
//  * table path (16-bit perm inside the record image): pj from a loop over the lanes that may have a
//    later equal j (512-entry hashed max-table, candidates verified exactly with readlane); writes
//    perm[i_t] = F_t and perm[j_t] = V_t unless a later lane rewrites j_t or j_t is a later i.
// Tables are tagged with a per-wave chunk counter (stab[MFG_STAB_CTR]) so they are never cleared.
// Returns j of the first accepted draw (i == hi), used by empty_positions().pop().
template <typename PT>
__device__ int mt_randbelow_seq(const Env& e, int hi, int lo, PT* perm) {
  uint32_t* mt = e.mt();
  const int lane = e.lane;
  int idx = e.H(H_MT_IDX);
  int icur = hi;
  int first_j = -1;
  uint32_t* ptab = e.stab;                    // [64] rank -> tag | max lane with j == i_rank
  uint32_t* htab = e.stab + MFG_STAB_PTAB;    // [MFG_STAB_HASH] j-hash -> tag | max lane
  const bool xchg = sizeof(PT) == 4 && e.S->xchg_ordered;
  uint32_t ctr = perm ? (uint32_t)uni((int)e.stab[MFG_STAB_CTR]) : 0u;
  while (icur >= lo) {
    if (idx >= 624) {
      mt_twist(e);
      idx = 0;
    }
    const int lmax = 624 - idx;
    const bool has = lane < lmax;
    // lanes past the state read the words after it (perm / scratch, inside the slice) and are discarded
    const uint32_t y = mt_temper(mt[idx + lane]);
    int A;
    u64 accm;
    int il;
    uint32_t r;
    bool act, acc;
    if (icur - 63 >= lo && 32 - __clz(icur + 1) == 32 - __clz(icur - 62)) {
      // fast path: every lane's i is >= lo and bitlen(i+1) is the same for the whole chunk, so
      // r_l = y_l >> (32 - k) is fixed and accept_l <=> A_l <= c_l = icur - r_l
      r = y >> __clz(icur + 1);
      const int c = has ? icur - (int)r : -1;
      A = mbcnt(ballot(c >= 63));  // lower bound: the lanes that accept whatever precedes them
      for (;;) {
        accm = ballot(A <= c);
        const int An = mbcnt(accm);
        if (!ballot(An != A)) break;
        A = An;
      }
      il = icur - A;
      acc = A <= c;
      act = has;
    } else {
      A = lane;
      for (;;) {
        il = icur - A;
        act = has && il >= lo;
        uint32_t n = act ? (uint32_t)(il + 1) : 2u;
        int k = 32 - __clz((int)n);
        r = act ? (y >> (32 - k)) : 0u;
        acc = act && r <= (uint32_t)il;
        accm = ballot(acc);
        int An = mbcnt(accm);
        if (!ballot(An != A)) break;
        A = An;
      }
    }
    const int consumed = popc(ballot(act));
    const int nacc = popc(accm);
    if (first_j < 0 && nacc) first_j = rl((int)r, ffs64(accm));
    if (perm && nacc) {
      const int i = acc ? il : icur, j = acc ? (int)r : icur;
      const int P0i = perm[i];
      ctr++;  // tables are zeroed at kernel start; < 2^26 chunks per launch
      const uint32_t tag = ctr << 6;
      const int imin = icur - nacc + 1;
      if (acc && j >= imin && j != i) atomicMax(&ptab[icur - j], tag | (uint32_t)lane);
      if (xchg) {
        wave_sync();
        const uint32_t tp = ptab[A & 63];
        int ptr = (acc && (tp >> 6) == ctr) ? (int)(tp & 63u) : -1;
        int v = P0i;
        while (ballot(ptr >= 0)) {
          const int src = ptr >= 0 ? ptr : lane;
          const int v2 = __shfl(v, src), p2 = __shfl(ptr, src);
          if (ptr >= 0) { v = v2; ptr = p2; }
        }
        int F = 0;
        if (acc) F = (int)atomicExch((uint32_t*)&perm[j], (uint32_t)v);
        wave_sync();
        if (acc) perm[i] = (PT)F;
        wave_sync();
      } else {
        const int P0j = perm[j];
        const int hj = j & (MFG_STAB_HASH - 1);
        if (acc) atomicMax(&htab[hj], tag | (uint32_t)lane);
        wave_sync();
        const uint32_t th = htab[hj], tp = ptab[A & 63];
        const bool cand = acc && (int)(th & 63u) != lane;  // some later lane shares j's hash
        int pj = -1;
        u64 later = 0;
        u64 nm = ballot(cand);
        while (nm) {
          const int s2 = ffs64(nm);
          nm &= nm - 1;
          const bool eq = acc && rl(j, s2) == j;
          if (eq && s2 < lane) pj = s2;
          if (ballot(eq && lane > s2)) later |= 1ull << s2;
        }
        int ptr = (acc && (tp >> 6) == ctr) ? (int)(tp & 63u) : -1;
        int v = P0i;
        while (ballot(ptr >= 0)) {
          const int src = ptr >= 0 ? ptr : lane;
          const int v2 = __shfl(v, src), p2 = __shfl(ptr, src);
          if (ptr >= 0) { v = v2; ptr = p2; }
        }
        const int Vj = __shfl(v, pj >= 0 ? pj : lane);
        const int F = pj >= 0 ? Vj : P0j;
        if (acc) perm[i] = (PT)F;
        if (acc && !((later >> lane) & 1) && !(j >= imin && j < i)) perm[j] = (PT)v;
        wave_sync();
      }
    }
    icur -= nacc;
    idx += consumed;
  }
  if (perm && lane == 0) e.stab[MFG_STAB_CTR] = ctr;
  e.setH(H_MT_IDX, idx);
  wave_sync();
  return first_j;
}

// 16-bit exchange in LDS: ds_mskor_rtn_b32 (MEM = (MEM & ~mask) | data, returns the old word) on the
// aligned word holding `p`, so a floor permutation can stay u16 in LDS. Conflicting lanes of one
// instruction are applied in lane order (probed by mfg_create, k_probe_xchg).
__device__ __forceinline__ uint32_t lds_xchg_u16(uint16_t* p, uint32_t v) {
  const uint32_t a = (uint32_t)(uintptr_t)p;  // low 32 bits of a generic LDS address = the LDS offset
  const uint32_t sh = (a & 2u) << 3;
  const uint32_t mask = 0xFFFFu << sh, data = (v & 0xFFFFu) << sh;
  uint32_t old;
  asm volatile("ds_mskor_rtn_b32 %0, %1, %2, %3\n\ts_waitcnt lgkmcnt(0)"
               : "=v"(old)
               : "v"(a & ~3u), "v"(mask), "v"(data)
               : "memory");
  return (old >> sh) & 0xFFFFu;
}
// The same exchange split in two: issue (returns the raw old dword, not yet waited for), then wait
// (tied to that value, so nothing reads it early) and extract the 16-bit half. LDS operations complete
// in issue order, so the compiler's own counted lgkmcnt waits stay conservative around it.
__device__ __forceinline__ uint32_t lds_xchg_u16_issue(uint16_t* p, uint32_t v) {  // v < 65536
  const uint32_t a = (uint32_t)(uintptr_t)p;
  const uint32_t sh = (a & 2u) << 3;
  const uint32_t mask = 0xFFFFu << sh, data = v << sh;
  uint32_t old;
  asm volatile("ds_mskor_rtn_b32 %0, %1, %2, %3" : "=v"(old) : "v"(a & ~3u), "v"(mask), "v"(data) : "memory");
  return old;
}
__device__ __forceinline__ uint32_t lds_xchg_u16_wait(uint32_t old, uint16_t* p) {
  asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(old) : : "memory");
  const uint32_t sh = ((uint32_t)(uintptr_t)p & 2u) << 3;
  return (old >> sh) & 0xFFFFu;
}

// k_replay's shuffle: the exchange path of mt_randbelow_seq specialised for the replay kernel (64
// draws per chunk, the record's own u16 permutation, 16-bit exchanges). Out-of-play lanes read and write a per-lane sink word instead of
// branching, so a block runs without exec-mask changes.
// stab: [64] rank table (tag << 6 | lane), [64] chunk counter
#define RP_CTR 64
#define RP_STAB_N 65
#define RP_HDR_N 8  // header ints k_replay keeps in its slice (H_DEBT, H_MT_IDX)
static_assert(H_DEBT < RP_HDR_N && H_MT_IDX < RP_HDR_N, "k_replay header slice");
#ifndef RP_SERIAL_FWD
#define RP_SERIAL_FWD 4  // blocks with at most this many forwards resolve them serially (no LDS table)
#endif
// The chunk's acceptance fixed point: from the seed m, iterate m = ballot(mbcnt(m) <= c) until it is stable;
// returns A = mbcnt(m) (#accepted lanes below this one) and leaves the accepted set in m.
__device__ __forceinline__ int accept_ranks(u64& m, int c) {
  for (;;) {
    const int A = mbcnt(m);
    const u64 m2 = ballot(A <= c);
    if (m2 == m) return A;
    m = m2;
  }
}
// TOP14: every width k = bitlen(i + 1) is <= 14 (nf < 16384), so r = y >> (32 - k) reads only bits
// 18..31 of the tempered word, which the last tempering step (y ^= y >> 18) leaves unchanged.
// SWAP = false: the draws of a shuffle of hi + 1 elements only (randbelow(i + 1) for i = hi .. 1, no
// permutation), e.g. shuffle(empty_positions) in the reset, on the same chunked path.
// Returns j of the first accepted draw (i == hi) when SWAP is false (random.shuffle(list); list.pop() takes it).
template <bool TOP14, bool SWAP = true>
__device__ int replay_shuffle_t(const Env& e, uint16_t* perm, int hi) {
  uint32_t* mt = e.mt();
  const int lane = e.lane;
  int first_j = -1;
  // 128 B: one u16 per lane; lanes l and l + 32 share a dword: they sit in different lane groups of the exchange,
  // so the rejected lanes' sink edits of one group never hit the same dword
  uint16_t* sink = (uint16_t*)e.scratch + (((lane & 31) << 1) | (lane >> 5));
  uint32_t* ptab = e.stab;
  const int lo = 1;
  int idx = e.H(H_MT_IDX);
  int icur = hi;
  uint32_t ctr = SWAP ? (uint32_t)uni((int)e.stab[RP_CTR]) : 0u;
  // Every chunk reads 64 words. Near the end of the state (idx > 560) the lanes past word 623 compute
  // the next state's first words directly from the current one (new[i] = mix(mt[i], mt[i+1],
  // mt[i+397]) for i < 227, the twist's first phase), so a chunk may run past the end: idx then exceeds
  // 624 and the in-place twist that follows (idx -= 624) writes the same words. Away from the end
  // (idx <= 560) the raw words of the next chunk are loaded one chunk ahead, so whether this chunk's
  // words are already in yw follows from idx alone (a twisted state had idx >= 624 > 560).
  uint32_t yw = idx <= 560 ? mt[idx + lane] : 0u;
  const int lane34 = (3 * lane) >> 2;
  while (icur >= lo) {
    if (idx > 560) {
      if (idx >= 624) {
        mt_twist(e);
        idx -= 624;
      }
      const int jw = idx + lane;
      if (idx <= 560) {
        yw = mt[jw];
      } else {
        const int jn = jw >= 624 ? jw - 624 : 0;
        const uint32_t nw = mt_mix(mt[jn], mt[jn + 1], mt[jn + 397]);
        yw = jw < 624 ? mt[jw < 624 ? jw : 0] : nw;
      }
    }
    const uint32_t y = TOP14 ? mt_temper3(yw) : mt_temper(yw);
    // One bit width per chunk: k = bitlen(icur + 1), and the chunk stops where bitlen(i + 1) would
    // change (i < 2^(k-1) - 1) or at lo. Within it accept <=> A <= c = min(icur - r, span), with
    // r = y >> (32 - k) fixed per lane, and lanes whose A exceeds span are not consumed (their words
    // start the next chunk). So every chunk takes the same branch-free path, power-of-two crossings
    // and the i < 64 tail included.
    const int sh = __clz(icur + 1);
    const int span = icur - max(lo, (int)(0x80000000u >> sh) - 1);  // highest rank at width k
    uint32_t r = y >> sh;
    const int c = min(icur - (int)r, span);
    // A_l = #accepted lanes < l: Jacobi iteration from a seed at A_l ~ 3l/4 (the mean acceptance; 1.91 rounds per
    // chunk instead of 2.15 from the sure lower bound c_l >= l, simulated over C3's chunks). Any seed converges to
    // the same unique fixed point (lane l is exact after l rounds).
    u64 m = ballot(c >= lane34);
    const int A = accept_ranks(m, c);
    const int nacc = popc(m);
    // ranks are monotone in the lane: all 64 words are consumed unless the band fills (nacc = span + 1), and then
    // exactly the lanes up to the last accepted one (scalar, no vector compare)
    const int consumed = nacc > span ? 64 - __builtin_clzll(m) : 64;
    const int inext = icur - nacc, idxn = idx + consumed;
    if constexpr (!SWAP) {
      if (first_j < 0 && m) first_j = rl((int)r, ffs64(m));
      if (idxn <= 560) yw = mt[idxn + lane];
    } else {
    // (a chunk with no accepted draw runs the block on the sinks: rare, and one branch less per chunk)
    const bool acc = lanes(m);
    const int i = icur - A, j = (int)r;
    // every lane reads its i cell: rejected lanes read the next accepted rank's cell (the same address as that
    // lane: a broadcast, no sink bank); only accepted lanes write it back
    uint16_t* pi = perm + i;
    int v = (int)*pi;
    // V_t (value leaving i_t): if earlier draws s < t moved a value onto i_t (j_s == i_t, i.e. j_s in
    // the block's own i range (inext, i)), the last one's V_s. Rare at large i: a single scalar test
    // skips it. Few forwards: walk them in ascending s, so V_s is final before it is forwarded to rank
    // icur - j_s (rejected lanes sharing that rank carry no swap and may take the value harmlessly).
    // Many (small i): a rank table (tag | lane, keyed by icur - j) gives each draw its forward source
    // and pointer jumping resolves the chains.
    u64 cm = ballot(j > inext) & ballot(j < i) & m;
    if (cm) {
      if (popc(cm) <= RP_SERIAL_FWD) {
        const int keyv = icur - j;  // the rank whose i equals this lane's j
        do {
          const int s = ffs64(cm);
          asm volatile("s_bitset0_b64 %0, %1" : "+s"(cm) : "s"(s));
          const int key = rl(keyv, s);
          const int vs = rl(v, s);
          v = A == key ? vs : v;
        } while (cm);
      } else {
        const bool fwd = lanes(cm);
        ctr++;  // tables are zeroed at kernel start; < 2^26 chunks per launch
        const uint32_t tag = ctr << 6;
        atomicMax(&ptab[fwd ? icur - j : lane], fwd ? tag | (uint32_t)lane : 0u);  // max with 0: no-op
        wave_sync();
        const uint32_t tp = ptab[A & 63];
        int ptr = (acc && (tp >> 6) == ctr) ? (int)(tp & 63u) : -1;
        while (ballot(ptr >= 0)) {
          const int src = ptr >= 0 ? ptr : lane;
          const int v2 = __shfl(v, src), p2 = __shfl(ptr, src);
          if (ptr >= 0) { v = v2; ptr = p2; }
        }
      }
    }
    // F = value landing on i: the exchange returns the previous same-address draw's V or P0[j]. The 16-bit half's
    // shift comes from j: shifts read the low 5 bits, so j << 4 is (j & 1) * 16 (perm is dword aligned in every LDS
    // image); rejected lanes edit either half of their sink word. The next chunk's MT words are loaded while the
    // exchange is in flight.
    uint32_t F;
    {
      const uint32_t sh = (uint32_t)j << 4;
      const uint32_t ad = (uint32_t)(uintptr_t)(acc ? &perm[j] : sink) & ~3u;
      asm volatile("ds_mskor_rtn_b32 %0, %1, %2, %3" : "=v"(F) : "v"(ad), "v"(0xFFFFu << (sh & 31u)),
                   "v"((uint32_t)v << (sh & 31u)) : "memory");
      if (idxn <= 560) yw = mt[idxn + lane];
      asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(F) : : "memory");
      asm("v_lshrrev_b32 %0, %1, %2" : "=v"(F) : "v"(sh), "v"(F));  // low 5 bits of sh; the i write keeps 16 bits
    }
    if (acc) *pi = (uint16_t)F;
    wave_sync();
    }
    icur = inext;
    idx = idxn;
  }
  if (idx > 624) {  // words of the next state were consumed: make the state canonical (CPython's mti)
    mt_twist(e);
    idx -= 624;
  }
  if (SWAP && lane == 0) e.stab[RP_CTR] = ctr;
  e.setH(H_MT_IDX, idx);
  wave_sync();
  return first_j;
}
__device__ __forceinline__ void replay_shuffle(const Env& e, uint16_t* perm) {
  if (e.S->replay_top14) replay_shuffle_t<true>(e, perm, e.S->nf - 1);
  else replay_shuffle_t<false>(e, perm, e.S->nf - 1);
}

// ---- two-wave replay (large floor lists: the 1-wave replay slice leaves <= 2 waves per SIMD) ----------------
// The draws of a shuffle (MT words, tempering, acceptance) never read the permutation, so one wave (the
// producer) runs them ahead for all of an env's debt while a second wave (the consumer) applies the swap blocks:
// per chunk the producer writes (icur, nacc) and the accepted draws' j in rank order to a ring in LDS; the two
// waves meet at one workgroup barrier per RP2_R chunks (double-buffered ring). Exactly the single-wave
// replay's arithmetic: the producer is replay_shuffle_t's draw half, the consumer its swap half with lane = rank.
#define RP2_R 16                       // chunks per ring half
#define RP2_REC (4 + 2 * MFG_WAVE)     // bytes per chunk record: icur | nacc << 16, then j[64] (u16)
#define RP2_RING (2 * RP2_R * RP2_REC + 16)  // both halves + [0] per-half chunk count x 2, [2] done phase
struct Rp2Prod {  // producer state carried across ring phases
  int s, icur, idx;
  uint32_t yw;
};
template <bool TOP14>
__device__ void rp2_produce(const Env& e, uint8_t* half, int* cnt, Rp2Prod& st, int d, int hi) {
  uint32_t* mt = e.mt();
  const int lane = e.lane, lo = 1;
  int n = 0;
  while (n < RP2_R && st.s < d) {
    if (st.idx > 560) {
      if (st.idx >= 624) {
        mt_twist(e);
        st.idx -= 624;
      }
      const int jw = st.idx + lane;
      if (st.idx <= 560) {
        st.yw = mt[jw];
      } else {
        const int jn = jw >= 624 ? jw - 624 : 0;
        const uint32_t nw = mt_mix(mt[jn], mt[jn + 1], mt[jn + 397]);
        st.yw = jw < 624 ? mt[jw < 624 ? jw : 0] : nw;
      }
    }
    const int icur = st.icur;
    const uint32_t y = TOP14 ? mt_temper3(st.yw) : mt_temper(st.yw);
    const int sh = __clz(icur + 1);
    const int span = icur - max(lo, (int)(0x80000000u >> sh) - 1);
    const uint32_t r = y >> sh;
    const int c = min(icur - (int)r, span);
    u64 m = ballot(c >= (3 * lane) >> 2);  // the single-wave replay's seed and consumed count (replay_shuffle_t)
    const int A = accept_ranks(m, c);
    const int nacc = popc(m);
    const int consumed = nacc > span ? 64 - __builtin_clzll(m) : 64;
    uint8_t* rec = half + n * RP2_REC;
    if (lanes(m)) ((uint16_t*)(rec + 4))[A] = (uint16_t)r;
    if (lane == 0) *(int*)rec = icur | (nacc << 16);
    const int idxn = st.idx + consumed;
    if (idxn <= 560) st.yw = mt[idxn + lane];
    st.idx = idxn;
    st.icur = icur - nacc;
    n++;
    if (st.icur < lo) {  // this shuffle is done: the next one starts at the top
      st.s++;
      st.icur = hi;
    }
  }
  if (lane == 0) *cnt = n;
}
__device__ void rp2_consume(const Env& e, const uint8_t* half, int n, uint32_t& ctr) {
  uint16_t* perm = e.perm();
  const int lane = e.lane;
  uint16_t* sink = (uint16_t*)e.scratch + lane;
  uint32_t* ptab = e.stab;
  // the half's chunk headers, lane q = chunk q (read per chunk with v_readlane, off the LDS chain)
  const int hds = lane < n ? *(const int*)(half + lane * RP2_REC) : 0;
  for (int q = 0; q < n; q++) {
    const uint8_t* rec = half + q * RP2_REC;
    const int hd = rl(hds, q);
    const int icur = hd & 0xFFFF, nacc = hd >> 16;
    if (!nacc) continue;
    const bool acc = lane < nacc;
    const int A = lane;
    // j and the value leaving i are read together (one LDS round trip)
    const int jraw = (int)((const uint16_t*)(rec + 4))[lane];
    uint16_t* const ptop = perm + icur;
    uint16_t* pi = ptop - min(A, nacc);  // lanes past the block read the next block's top (a broadcast)
    int v = (int)*pi;
    const int j = acc ? jraw : icur;
    const int i = icur - A, inext = icur - nacc;
    const u64 m = ballot(acc);
    u64 cm = ballot(j > inext) & ballot(j < i) & m;
    if (cm) {
      if (popc(cm) <= RP_SERIAL_FWD) {
        const int keyv = icur - j;
        do {
          const int s2 = ffs64(cm);
          asm volatile("s_bitset0_b64 %0, %1" : "+s"(cm) : "s"(s2));
          const int key = rl(keyv, s2);
          const int vs = rl(v, s2);
          v = A == key ? vs : v;
        } while (cm);
      } else {
        const bool fwd = lanes(cm);
        ctr++;
        const uint32_t tag = ctr << 6;
        atomicMax(&ptab[fwd ? icur - j : lane], fwd ? tag | (uint32_t)lane : 0u);
        wave_sync();
        const uint32_t tp = ptab[A & 63];
        int ptr = (acc && (tp >> 6) == ctr) ? (int)(tp & 63u) : -1;
        while (ballot(ptr >= 0)) {
          const int src = ptr >= 0 ? ptr : lane;
          const int v2 = __shfl(v, src), p2 = __shfl(ptr, src);
          if (ptr >= 0) { v = v2; ptr = p2; }
        }
      }
    }
    uint32_t F = lds_xchg_u16_issue(acc ? &perm[j] : sink, (uint32_t)v);
    F = lds_xchg_u16_wait(F, acc ? &perm[j] : sink);
    if (acc) *pi = (uint16_t)F;
    wave_sync();
  }
}

// random.shuffle(Entities._floor_positions) (global_entities.py:47-55)
template <typename PT>
__device__ __forceinline__ void floor_shuffle_t(const Env& e, PT* perm) {
  if constexpr (sizeof(PT) == 2) {
    if (e.S->xchg_ordered) {  // the branch-free exchange path (the replay kernel's) whenever it is probed
      replay_shuffle(e, perm);
      return;
    }
  }
  mt_randbelow_seq(e, e.S->nf - 1, 1, perm);
}
__device__ __forceinline__ void floor_shuffle(const Env& e) { floor_shuffle_t(e, e.perm()); }

// Pay the shuffle debt accumulated by membership-only floorlist calls (check_pos_validity, Q3).
template <typename PT>
__device__ void pay_debt_t(const Env& e, PT* perm) {
  int debt = e.H(H_DEBT);
  for (int k = 0; k < debt; k++) floor_shuffle_t(e, perm);
  e.setH(H_DEBT, 0);
  wave_sync();
}
__device__ __forceinline__ void pay_debt(const Env& e) { pay_debt_t(e, e.perm()); }

// CPython random.seed(int) -> init_by_array (Modules/_randommodule.c); serial, once per env
__device__ void mt_seed(const Env& e, const uint32_t* key, int len) {
  uint32_t* mt = e.mt();
  if (e.lane == 0) {
    mt[0] = 19650218u;
    for (int i = 1; i < 624; i++) mt[i] = 1812433253u * (mt[i - 1] ^ (mt[i - 1] >> 30)) + (uint32_t)i;
    int i = 1, j = 0;
    int k = 624 > len ? 624 : len;
    for (; k; k--) {
      mt[i] = (mt[i] ^ ((mt[i - 1] ^ (mt[i - 1] >> 30)) * 1664525u)) + key[j] + (uint32_t)j;
      i++; j++;
      if (i >= 624) { mt[0] = mt[623]; i = 1; }
      if (j >= len) j = 0;
    }
    for (k = 623; k; k--) {
      mt[i] = (mt[i] ^ ((mt[i - 1] ^ (mt[i - 1] >> 30)) * 1566083941u)) - (uint32_t)i;
      i++;
      if (i >= 624) { mt[0] = mt[623]; i = 1; }
    }
    mt[0] = 0x80000000u;
  }
  e.setH(H_MT_IDX, 624);
  wave_sync();
}

// ------------------------------------------------------------------------------------------------
// numpy PCG64 (XSL-RR 128/64) + Generator.uniform — state in LDS (4 x u64: state hi, lo, inc hi, lo)
// ------------------------------------------------------------------------------------------------
__device__ double pcg_uniform(const Env& e, double lo, double hi) {
  uint64_t* p = e.pcg();
  unsigned __int128 st = ((unsigned __int128)p[0] << 64) | p[1];
  const unsigned __int128 inc = ((unsigned __int128)p[2] << 64) | p[3];
  const unsigned __int128 mult = ((unsigned __int128)2549297995355413924ULL << 64) | 4865540595714422341ULL;
  st = st * mult + inc;
  const uint64_t h = (uint64_t)(st >> 64), l = (uint64_t)st;
  const unsigned rot = (unsigned)(h >> 58);
  const uint64_t x = h ^ l;
  const uint64_t out = (x >> rot) | (x << ((64 - rot) & 63));
  wave_sync();
  if (e.lane == 0) { p[0] = (uint64_t)(st >> 64); p[1] = (uint64_t)st; }
  wave_sync();
  const double u = (double)(out >> 11) * (1.0 / 9007199254740992.0);
  return lo + (hi - lo) * u;
}

// ------------------------------------------------------------------------------------------------
// Philox4x32-10 (synthetic actions for fused rollouts): key (seed, env), counter (step, agent, 0, 0)
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t philox_u32(uint32_t k0, uint32_t k1, uint32_t c0, uint32_t c1) {
  uint32_t c2 = 0, c3 = 0;
#pragma unroll
  for (int r = 0; r < 10; r++) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
    const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0, n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
    c1 = (uint32_t)p1;
    c3 = (uint32_t)p0;
    c0 = n0;
    c2 = n2;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c0;
}

// ------------------------------------------------------------------------------------------------
// entity model queries (global pos_dict semantics, groups/objects.py:193-214)
// ------------------------------------------------------------------------------------------------
enum { K_NONE = -1, K_DOOR = 1, K_ITEM = 3, K_POD = 4, K_DROP = 5, K_DIRT = 6, K_DEST = 7, K_MACHINE = 8, K_MAINT = 9,
       K_WALL = 15 };  // K_WALL: id-collision pair code only (the wall is identified by its cell)

// ballot of group slots at `cell` whose word has all bits of `need`
__device__ __forceinline__ u64 grp_at(const int* tbl, int n, int cell, int need, int lane) {
  int w = lane < n ? tbl[lane] : 0;
  return ballot(lane < n && EW_POS(w) == cell && (w & need) == need);
}
// groups longer than a wave (dirt piles): lowest matching slot / number of matching slots, 64 per pass
__device__ __forceinline__ int grp_first(const int* tbl, int n, int cell, int need, int lane) {
  for (int b = 0; b < n; b += MFG_WAVE) {
    const u64 m = grp_at(tbl + b, n - b, cell, need, lane);
    if (m) return b + ffs64(m);
  }
  return -1;
}
__device__ __forceinline__ int grp_count(const int* tbl, int n, int cell, int need, int lane) {
  int c = 0;
  for (int b = 0; b < n; b += MFG_WAVE) c += popc(grp_at(tbl + b, n - b, cell, need, lane));
  return c;
}
// Agent- and door-parallel code runs NW passes of 64 lanes (NW = 2: specs with more than 64 agents or doors); in pass h
// lane l holds agent / door h * 64 + l. NW is a template parameter of the step and reset kernels
// (MfgDevSpec::lane_passes).
// number of agents at `cell`
template <int NW>
__device__ __forceinline__ int agents_count_at(const Env& e, int cell) {
  const int A = e.S->A;
  int n = 0;
#pragma unroll
  for (int h = 0; h < NW; h++) {
    const int a = h * MFG_WAVE + e.lane;
    const int p = a < A ? e.agpos()[a] : -1;
    n += popc(ballot(a < A && p == cell));
  }
  return n;
}
__device__ __forceinline__ int door_idx(const Env& e, int cell) {
  int d = e.S->door_of[cell];
  return d == 0xFF ? -1 : d;
}
// the present int-identifier entity at `cell` whose identifier equals `id` (at most one, pos_dict keeps
// identifiers unique per cell); returns its kind, *slot = group slot
__device__ int find_present_id(const Env& e, int cell, int id, int* slot) {
  const int lane = e.lane;
  int d = door_idx(e, cell);
  if (d >= 0 && d == id && (e.door()[d] & DW_PRESENT)) { *slot = d; return K_DOOR; }
  u64 m;
  int base = e.H(H_ITEM_BASE);
  m = grp_at(e.items(), e.H(H_N_ITEMS), cell, EW_PRESENT, lane) & ballot(base + lane == id);
  if (m) { *slot = ffs64(m); return K_ITEM; }
  base = e.H(H_POD_BASE);
  m = grp_at(e.pods(), e.H(H_N_PODS), cell, EW_PRESENT, lane) & ballot(base + lane == id);
  if (m) { *slot = ffs64(m); return K_POD; }
  base = e.H(H_DROP_BASE);
  m = grp_at(e.drops(), e.H(H_N_DROPS), cell, EW_PRESENT, lane) & ballot(base + lane == id);
  if (m) { *slot = ffs64(m); return K_DROP; }
  base = e.H(H_DEST_BASE);
  m = grp_at(e.dests(), e.H(H_N_DESTS), cell, EW_PRESENT, lane) & ballot(base + lane == id);
  if (m) { *slot = ffs64(m); return K_DEST; }
  const int nd = e.H(H_N_DIRT);
  for (int b = 0; b < nd; b += MFG_WAVE) {
    const int i = b + lane;
    m = grp_at(e.dirtpos() + b, nd - b, cell, EW_PRESENT, lane) & ballot(i < nd && e.dirtid()[i < nd ? i : 0] == id);
    if (m) { *slot = b + ffs64(m); return K_DIRT; }
  }
  if (e.S->mmax) {
    base = e.H(H_MACHINE_BASE);
    m = grp_at(e.machines(), e.H(H_N_MACHINES), cell, EW_PRESENT, lane) & ballot(base + lane == id);
    if (m) { *slot = ffs64(m); return K_MACHINE; }
  }
  if (e.S->kmax) {
    base = e.H(H_MAINT_BASE);
    m = grp_at(e.maints(), e.H(H_N_MAINTS), cell, EW_PRESENT, lane) & ballot(base + lane == id);
    if (m) { *slot = ffs64(m); return K_MAINT; }
  }
  return K_NONE;
}
// Objects.notify_del_entity x2 on the global pos_dict: list.remove() drops the first identifier-equal entry
__device__ void global_remove_id(const Env& e, int cell, int id) {
  int slot;
  int k = find_present_id(e, cell, id, &slot);
  if (e.lane == 0) {
    switch (k) {
      case K_DOOR: e.door()[slot] &= ~DW_PRESENT; break;
      case K_ITEM: e.items()[slot] &= ~EW_PRESENT; break;
      case K_POD: e.pods()[slot] &= ~EW_PRESENT; break;
      case K_DROP: e.drops()[slot] &= ~EW_PRESENT; break;
      case K_DEST: e.dests()[slot] &= ~EW_PRESENT; break;
      case K_DIRT: e.dirtpos()[slot] &= ~EW_PRESENT; e.hdrp[H_DIRT_TOUCH] = 1; break;
      case K_MACHINE: e.machines()[slot] &= ~EW_PRESENT; break;
      case K_MAINT: e.maints()[slot] &= ~EW_PRESENT; break;
      default: break;
    }
  }
  wave_sync();
}
__device__ __forceinline__ bool present_closed_door(const Env& e, int cell) {
  int d = door_idx(e, cell);
  if (d < 0) return false;
  int w = e.door()[d];
  return (w & DW_PRESENT) && !(w & DW_OPEN);
}
// any entity blocking the position (states.py:259-270): walls, closed doors, blocking agents
template <int NW>
__device__ bool blocked_at(const Env& e, int cell) {
  if (e.S->level[cell] == 1) return true;
  if (present_closed_door(e, cell)) return true;
  const int A = e.S->A;
  u64 m = 0;
#pragma unroll
  for (int h = 0; h < NW; h++) {
    const int a = h * MFG_WAVE + e.lane;
    m |= ballot(a < A && e.agpos()[a < A ? a : 0] == cell && e.S->s.agent_blocking[a < A ? a : 0]);
  }
  return m != 0;
}
// present maintainers at cell (colliders, maintenance/groups.py:11-13)
__device__ __forceinline__ u64 maints_at(const Env& e, int cell) {
  return e.S->kmax ? grp_at(e.maints(), e.H(H_N_MAINTS), cell, EW_PRESENT, e.lane) : 0ull;
}
// number of colliders in the global list at cell (walls, closed doors, agents, maintainers)
template <int NW>
__device__ int colliders_at(const Env& e, int cell) {
  int n = (e.S->level[cell] == 1) + (present_closed_door(e, cell) ? 1 : 0);
  return n + agents_count_at<NW>(e, cell) + popc(maints_at(e, cell));
}

// Per door (pass h, lane l: door h * 64 + l, counts of doors >= nd are 0): the number of entities in the global
// pos_dict at its cell (all: Door.tick's len(pos_dict), doors/entitites.py:109) or of its colliders (coll:
// colliders_at), by one lane-parallel LDS histogram per entity table instead of a uniform loop over every table per
// door. cnt: >= 64 NW ints of LDS scratch.
template <int NW>
__device__ void door_cell_counts(const Env& e, int* cnt, bool coll, int (&out)[NW]) {
  SpecP S = e.S;
  const int lane = e.lane, nd = S->nd, HW = S->HW;
#pragma unroll
  for (int h = 0; h < NW; h++) {
    const int d = h * MFG_WAVE + lane;
    if (d < nd) {
      const int w = e.door()[d];
      cnt[d] = coll ? ((w & DW_PRESENT) && !(w & DW_OPEN) ? 1 : 0) : ((w & DW_PRESENT) ? 1 : 0);
    }
  }
  wave_sync();
  auto add = [&](int cell) {  // cell < 0 or off-grid: nothing
    const int d = ((unsigned)cell < (unsigned)HW) ? S->door_of[cell] : 0xFF;
    if (d != 0xFF) atomicAdd(&cnt[d], 1);
  };
#pragma unroll
  for (int h = 0; h < NW; h++)
    if (h * MFG_WAVE + lane < S->A) add(e.agpos()[h * MFG_WAVE + lane]);
  auto grp = [&](const int* tbl, int n) {
    for (int i = lane; i < n; i += MFG_WAVE) {
      const int w = tbl[i];
      if (w & EW_PRESENT) add(EW_POS(w));
    }
  };
  if (!coll) {
    grp(e.items(), e.H(H_N_ITEMS));
    grp(e.pods(), e.H(H_N_PODS));
    grp(e.drops(), e.H(H_N_DROPS));
    grp(e.dests(), e.H(H_N_DESTS));
    grp(e.dirtpos(), e.H(H_N_DIRT));
    if (S->mmax) grp(e.machines(), e.H(H_N_MACHINES));
  }
  if (S->kmax) grp(e.maints(), e.H(H_N_MAINTS));
  wave_sync();
#pragma unroll
  for (int h = 0; h < NW; h++) out[h] = h * MFG_WAVE + lane < nd ? cnt[h * MFG_WAVE + lane] : 0;
  wave_sync();
}

// ------------------------------------------------------------------------------------------------
// spawn-position queries (global_entities.py:77-121)
// ------------------------------------------------------------------------------------------------
// a cell in the global list with no collider and no blocker (free_positions_generator)
__device__ __forceinline__ bool lane_cell_free(const Env& e, int cell) {
  if (present_closed_door(e, cell)) return false;
  const int A = e.S->A;
  for (int b = 0; b < A; b++)
    if (e.agpos()[b] == cell) return false;
  const int nk = e.S->kmax ? e.H(H_N_MAINTS) : 0;
  for (int i = 0; i < nk; i++) { int w = e.maints()[i]; if (EW_POS(w) == cell && (w & EW_PRESENT)) return false; }
  return true;
}
// first n free cells of a fresh floor shuffle -> out[0..k) (LDS scratch), returns k
__device__ int free_positions(const Env& e, int n, int* out) {
  floor_shuffle(e);
  const uint16_t* perm = e.perm();
  const int nf = e.S->nf;
  int k = 0;
  for (int b = 0; b < nf && k < n; b += MFG_WAVE) {
    int i = b + e.lane;
    int cell = i < nf ? (int)perm[i] : -1;
    bool f = i < nf && lane_cell_free(e, cell);
    u64 m = ballot(f);
    int rank = k + mbcnt(m);
    if (f && rank < n) out[rank] = cell;
    k += popc(m);
  }
  wave_sync();
  return k < n ? k : n;
}
__device__ int spawn_positions(const Env& e, int n, int ignore_blocking, int* out) {
  if (ignore_blocking) {  // floorlist[:n] (collection.py:368-369)
    floor_shuffle(e);
    int k = n < e.S->nf ? n : e.S->nf;
    for (int i = e.lane; i < k; i += MFG_WAVE) out[i] = e.perm()[i];
    wave_sync();
    return k;
  }
  return free_positions(e, n, out);
}

// ------------------------------------------------------------------------------------------------
// spawning (collection.py:102-151 and the group overrides)
// ------------------------------------------------------------------------------------------------
// append one int-id entity to a group table; it enters the global pos_dict only if no entity with an
// equal identifier is already there (Objects.notify_add_entity, objects.py:203-214)
__device__ void spawn_into(const Env& e, int* tbl, int hn, int base, int cell, int extra = 0) {
  int n = e.H(hn);
  int slot;
  int id = base + n;
  bool present = find_present_id(e, cell, id, &slot) == K_NONE;
  if (e.lane == 0) tbl[n] = cell | EW_ALIVE | (present ? EW_PRESENT : 0) | extra;
  e.setH(hn, n + 1);
  wave_sync();
}

__device__ double dirt_global_amount(const Env& e) {  // clean_up/groups.py:27-32: left-to-right sum
  double s = 0.0;
  const int n = e.H(H_N_DIRT);
  for (int i = 0; i < n; i++) s += e.dirtamt()[i];
  return s;
}

#define DIRTPILE_MAX_LOCAL 5.0  /* DirtPile(max_local_amount=5): the collection value is never forwarded (Q20) */

// DirtPiles.trigger_spawn (clean_up/groups.py:70-95); returns spawn_counter, *valid = result validity
__device__ int dirt_trigger_spawn(const Env& e, int q, double amount, int* valid, int* scratch) {
  const CS mfg_spec& s = e.S->s;
  double u = pcg_uniform(e, -s.dirt_n_var, s.dirt_n_var);
  int n_new = (int)fabs((double)q + u);
  pay_debt(e);
  int npos = free_positions(e, n_new, scratch);
  int n = npos < q ? npos : q;
  // amounts: drawn for range(q) before any placement (numpy PCG64); the first n are kept in scratch
  // after the positions (scratch_bytes is sized for both at the spec's largest spawn)
  double* amts = (double*)(scratch + ((n + 1) & ~1));
  for (int i = 0; i < q; i++) {
    double a = amount != 0.0 ? amount : s.dirt_initial_amount + pcg_uniform(e, -s.dirt_amount_var, s.dirt_amount_var);
    if (e.lane == 0 && i < n) amts[i] = a;
  }
  wave_sync();
  int counter = 0;
  for (int i = 0; i < n; i++) {
    const int cell = scratch[i];
    const double a = amts[i];
    if (dirt_global_amount(e) > s.dirt_max_global) { *valid = 0; return counter; }
    const int nd = e.H(H_N_DIRT);
    const int k = grp_first(e.dirtpos(), nd, cell, EW_ALIVE, e.lane);
    if (k >= 0) {
      double nv = e.dirtamt()[k] + a;
      wave_sync();
      if (e.lane == 0) {
        e.dirtamt()[k] = nv < DIRTPILE_MAX_LOCAL ? nv : DIRTPILE_MAX_LOCAL;
        e.hdrp[H_DIRT_TOUCH] = 1;
      }
      wave_sync();
    } else {
      if (nd >= e.S->dirt_cap) { e.setH(H_OVERFLOW, 1); *valid = 0; return counter; }
      int id = e.H(H_CNT_DIRT);
      int slot;
      bool present = find_present_id(e, cell, id, &slot) == K_NONE;
      if (e.lane == 0) {
        e.dirtpos()[nd] = cell | EW_ALIVE | (present ? EW_PRESENT : 0);
        e.dirtid()[nd] = id;
        e.dirtamt()[nd] = a;
        e.hdrp[H_DIRT_TOUCH] = 1;
      }
      e.setH(H_CNT_DIRT, id + 1);
      e.setH(H_N_DIRT, nd + 1);
      wave_sync();
      counter++;
    }
  }
  *valid = 1;
  return counter;
}

// remove dirt slot k keeping collection order (Collection.__delitem__)
__device__ void dirt_delete(const Env& e, int k) {
  const int nd = e.H(H_N_DIRT);
  const int cell = EW_POS(e.dirtpos()[k]);
  const int id = e.dirtid()[k];
  global_remove_id(e, cell, id);
  for (int b = k & ~(MFG_WAVE - 1); b < nd; b += MFG_WAVE) {  // shift slots k+1.. down by one, 64 per pass
    const int j = b + e.lane;
    const bool mv = j > k && j < nd;
    int p = 0, i = 0;
    double a = 0.0;
    if (mv) { p = e.dirtpos()[j]; i = e.dirtid()[j]; a = e.dirtamt()[j]; }
    wave_sync();
    if (mv) { e.dirtpos()[j - 1] = p; e.dirtid()[j - 1] = i; e.dirtamt()[j - 1] = a; }
    wave_sync();
  }
  e.setH(H_N_DIRT, nd - 1);
  e.setH(H_DIRT_TOUCH, 1);
  wave_sync();
}

// ------------------------------------------------------------------------------------------------
// step bookkeeping: rewards are accumulated per agent in the reference's result order
// ------------------------------------------------------------------------------------------------
template <int NW>
struct StepOut {
  double my_rew[NW];    // pass h, lane l: agent h * 64 + l's reward sum so far
  double g_rew;         // uniform: 'global' reward sum
  int my_act_ev[NW];    // per agent (as my_rew): act event bits
  int my_watch_ev[NW];  // per agent: watch event bits
  int my_slot[NW];      // per agent: action slot it executed this step, -1 if it did not act (paralyzed)
  u64 door_coll[NW];    // doors h * 64 + bit that received a WatchCollisions result
  u64 maint_coll;       // maintainers (collection slots) that received a WatchCollisions result
  int respawn_items_value, dirt_spawn_value, dirt_spawn_valid, door_autoclose, done_mask, dest_reached, crashed;
  int done;
};

// per-agent lane values (pass h, lane l = agent h * 64 + l): update agent a's entry (a uniform)
template <int NW, typename T>
__device__ __forceinline__ void agent_add(T (&v)[NW], int a, int lane, T x) {
#pragma unroll
  for (int h = 0; h < NW; h++)
    if (lane + h * MFG_WAVE == a) v[h] += x;
}
template <int NW, typename T>
__device__ __forceinline__ void agent_set(T (&v)[NW], int a, int lane, T x) {
#pragma unroll
  for (int h = 0; h < NW; h++)
    if (lane + h * MFG_WAVE == a) v[h] = x;
}
// agent a's entry of a per-agent lane value (a uniform)
template <int NW>
__device__ __forceinline__ int agent_get(const int (&v)[NW], int a) {
  return (NW == 1 || a < MFG_WAVE) ? rl(v[0], a & (MFG_WAVE - 1)) : rl(v[NW - 1], a & (MFG_WAVE - 1));
}
// bit d of a door / agent mask of NW words
template <int NW>
__device__ __forceinline__ void mask_set(u64 (&m)[NW], int d) {
  if (NW == 1 || d < MFG_WAVE) m[0] |= 1ull << (d & (MFG_WAVE - 1));
  else m[NW - 1] |= 1ull << (d & (MFG_WAVE - 1));
}
template <int NW>
__device__ __forceinline__ bool mask_get(const u64 (&m)[NW], int d) {
  return (((NW == 1 || d < MFG_WAVE) ? m[0] : m[NW - 1]) >> (d & (MFG_WAVE - 1))) & 1;
}
template <int NW>
__device__ __forceinline__ bool mask_any(const u64 (&m)[NW]) {
  u64 o = 0;
#pragma unroll
  for (int h = 0; h < NW; h++) o |= m[h];
  return o != 0;
}

__device__ const CS mfg_action& action_of(const Env& e, int a, int slot) { return e.S->s.actions[a][slot]; }

__device__ __forceinline__ void set_agent_pos(const Env& e, int a, int cell) {
  wave_sync();
  if (e.lane == 0) {
    e.agpos()[a] = cell;
    int c = e.hdr()[H_ARRIVAL];
    e.agarr()[a] = c;
    e.hdr()[H_ARRIVAL] = c + 1;
  }
  wave_sync();
}

// ------------------------------------------------------------------------------------------------
// actions (environment/actions.py, modules/*/actions.py)
// ------------------------------------------------------------------------------------------------
// DoorUse.do (doors/actions.py:18-34; get_entities_near_pos, global_entities.py:13-38): toggle every door
// present in the global pos_dict of the 3x3 around (x, y); valid if there was one
template <int NW>
__device__ bool door_use_at(const Env& e, int x, int y) {
  SpecP S = e.S;
  const int W = S->s.W;
  static const int MX[9] = {-1, 0, 1, -1, 0, 1, -1, 0, 1};
  static const int MY[9] = {-1, -1, -1, 0, 0, 0, 1, 1, 1};
  u64 toggle[NW];
#pragma unroll
  for (int h = 0; h < NW; h++) toggle[h] = 0;
  for (int k = 0; k < 9; k++) {
    const int px = x + MX[k], py = y + MY[k];
    if (px < 0 || py < 0 || px >= S->s.H || py >= W) continue;
    const int c = px * W + py;
    if (S->level[c] == 1) continue;
    const int d = door_idx(e, c);
    if (d >= 0 && (e.door()[d] & DW_PRESENT)) mask_set(toggle, d);
  }
  if (!mask_any(toggle)) return false;
  wave_sync();
#pragma unroll
  for (int h = 0; h < NW; h++) {
    const int d = h * MFG_WAVE + e.lane;
    if (d < S->nd && ((toggle[h] >> e.lane) & 1)) {
      int w = e.door()[d];
      if (w & DW_OPEN) w &= ~DW_OPEN;
      else w = (w & DW_PRESENT) | DW_OPEN | ((S->s.door_auto_close & 0xFF) << 8);
      e.door()[d] = w;
    }
  }
  wave_sync();
  return true;
}

template <int NW>
__device__ void do_action(const Env& e, StepOut<NW>& o, int a, int slot) {
  SpecP S = e.S;
  const CS mfg_action& ac = action_of(e, a, slot);
  const int op = ac.op;
  const int pos = uni(e.agpos()[a]);
  const int W = S->s.W;
  const int x = pos / W, y = pos % W;
  int valid = 0, coll = 0, aux = 0;
  if (op == MFG_ACT_NOOP) {
    valid = 1;
  } else if (op == MFG_ACT_MOVE) {  // actions.py:77-100, states.py:240-270, entity.py:175-199
    static const int DX[8] = {-1, -1, 0, 1, 1, 1, 0, -1};
    static const int DY[8] = {0, 1, 1, 1, 0, -1, -1, -1};
    const int nx = x + DX[ac.arg], ny = y + DY[ac.arg];
    const int t = nx * W + ny;  // levels are wall-bounded: a move never leaves the grid
    const bool blocked = blocked_at<NW>(e, t);
    int debt = 0;
    if (!blocked) debt++;  // check_pos_validity -> `pos in floorlist` shuffles (Q3)
    const bool not_blocked = !blocked && S->level[t] != 1;
    bool blocking_others = false;
    if (S->s.agent_blocking[a]) blocking_others = colliders_at<NW>(e, t) > 0 || blocked;  // is_occupied
    const bool v = pos != t && not_blocked && !blocking_others;
    if (v) {
      debt++;  // Entity.move re-checks validity (second shuffle)
      set_agent_pos(e, a, t);
      valid = 1;
      coll = colliders_at<NW>(e, t) > 1;
    } else {
      valid = 0;
      coll = 1;
    }
    e.setH(H_DEBT, e.H(H_DEBT) + debt);
    wave_sync();
  } else if (op == MFG_ACT_DOORUSE) {  // doors/actions.py:18-34
    valid = door_use_at<NW>(e, x, y);
  } else if (op == MFG_ACT_ITEM) {  // items/actions.py:41-63
    if (grp_at(e.drops(), e.H(H_N_DROPS), pos, EW_ALIVE, e.lane)) {
      valid = 0;  // inventories are always empty (pickup bug, Q8)
      aux = 1;
    } else {
      u64 m = grp_at(e.items(), e.H(H_N_ITEMS), pos, EW_ALIVE, e.lane);
      if (m) {
        const int k = ffs64(m);
        global_remove_id(e, pos, e.H(H_ITEM_BASE) + k);
        if (e.lane == 0) e.items()[k] = (e.items()[k] & ~0xFFFF) | EW_NOPOS;
        wave_sync();
        valid = 1;
      }
    }
  } else if (op == MFG_ACT_CHARGE) {  // batteries/actions.py:20-31, entitites.py:98-111
    if (grp_at(e.pods(), e.H(H_N_PODS), pos, EW_ALIVE, e.lane)) {
      const double ch = e.bat()[a];
      if (ch >= 1.0) valid = 0;
      else if (agents_count_at<NW>(e, pos) > 1) valid = 0;
      else {
        const double nv = S->s.pod_charge_rate + ch;
        wave_sync();
        if (e.lane == 0) e.bat()[a] = nv > 1.0 ? 1.0 : nv;
        wave_sync();
        valid = 1;
      }
    }
  } else if (op == MFG_ACT_CLEAN) {  // clean_up/actions.py:19-36
    const int k = grp_first(e.dirtpos(), e.H(H_N_DIRT), pos, EW_PRESENT, e.lane);
    if (k >= 0) {
      const double na = e.dirtamt()[k] - S->s.dirt_clean_amount;
      if (na <= 0) {
        dirt_delete(e, k);
      } else {
        wave_sync();
        if (e.lane == 0) {
          e.dirtamt()[k] = na < DIRTPILE_MAX_LOCAL ? na : DIRTPILE_MAX_LOCAL;
          e.hdrp[H_DIRT_TOUCH] = 1;
        }
        wave_sync();
      }
      valid = 1;
    }
  } else if (op == MFG_ACT_DEST) {  // destinations/actions.py:17-24
    if (grp_at(e.dests(), e.H(H_N_DESTS), pos, EW_ALIVE, e.lane)) {
      o.crashed = 1;  // AttributeError upstream (Q17)
      return;
    }
    valid = 0;
  }
  const double rw = aux ? (valid ? ac.aux0 : ac.aux1) : (valid ? ac.valid_reward : ac.fail_reward);
  agent_add(o.my_rew, a, e.lane, rw);
  agent_set(o.my_act_ev, a, e.lane, 0x80 | (valid ? 1 : 0) | (coll ? 2 : 0) | (aux ? 4 : 0));
}

// Agents act in list order (states.py:189-198), but most actions only depend on the agents before them
// through positions and door states: Noop, Move (no blocking agents in the spec), Charge, DoorUse, and an
// ItemAction on a cell without items or drop-offs (it fails). The leading run 0..F-1 of such agents is
// resolved lane-parallel (lane = agent); the ordered loop continues from the first other one (F):
//   * door state seen by agent a = initial state XOR the parity of the toggles of DoorUse agents b < a;
//   * cell occupancy seen by agent a = agents b < a at their new cells + agents b > a at their old ones;
//   * arrival order = the running counter + the exclusive count of earlier successful movers;
//   * floor-shuffle debt (Q3) = one per unblocked target + one per successful move, summed.
// Each agent's own reward terms keep their order (the action result is its first term).
// More than 64 agents (NW = 2): the run is resolved 64 agents at a time, each pass after the previous one's commit, so
// the agents of earlier passes are at their new cells (and their door toggles applied) in the record, and the agents
// of later passes at their old ones.
template <int NW>
__device__ int act_parallel(const Env& e, const int (&my_act)[NW], StepOut<NW>& o) {
  SpecP S = e.S;
  const int A = S->A, W = S->s.W, lane = e.lane;
  bool any_blocking = false;
#pragma unroll
  for (int h = 0; h < NW; h++) {
    const int al = h * MFG_WAVE + lane;
    any_blocking |= ballot(al < A && S->s.agent_blocking[al < A ? al : 0]) != 0;
  }
  // F: the first agent outside the lane-parallel class (classified before any pass: no action of the run changes
  // what the class depends on, the agent's own cell, slot and paralysis)
  int F = A;
  bool par_h[NW], ok_h[NW];
  int pos_h[NW];
#pragma unroll
  for (int h = NW - 1; h >= 0; h--) {
    const int al0 = h * MFG_WAVE + lane;
    const bool me = al0 < A;
    const int al = me ? al0 : 0;
    const bool par = me && e.agpar()[al] != 0;
    const bool ok_slot = me && my_act[h] >= 0 && my_act[h] < S->s.n_actions[al];
    const int op = ok_slot ? S->s.actions[al][my_act[h]].op : -1;
    const int pos = me ? e.agpos()[al] : -1;
    par_h[h] = par;
    ok_h[h] = ok_slot;
    pos_h[h] = pos;
    bool simple = !me || par;
    if (me && !par && ok_slot) {
      if (op == MFG_ACT_NOOP || op == MFG_ACT_CHARGE || op == MFG_ACT_DOORUSE) simple = true;
      else if (op == MFG_ACT_MOVE) simple = !any_blocking;
      else if (op == MFG_ACT_ITEM) {
        bool hit = false;
        const int ni = e.H(H_N_ITEMS), ndr = e.H(H_N_DROPS);
        for (int i = 0; i < ni; i++) { const int w = e.items()[i]; hit |= EW_POS(w) == pos && (w & EW_ALIVE); }
        for (int i = 0; i < ndr; i++) { const int w = e.drops()[i]; hit |= EW_POS(w) == pos && (w & EW_ALIVE); }
        simple = !hit;
      }
    }
    const u64 ns = ballot(!simple);
    if (ns) F = h * MFG_WAVE + ffs64(ns);
  }
  if (F == 0) return 0;
#pragma unroll
  for (int h = 0; h < NW; h++) {
    if (h * MFG_WAVE >= F) break;
    const int al0 = h * MFG_WAVE + lane;
    const bool me = al0 < A;
    const int al = me ? al0 : 0;
    const bool par = par_h[h];
    const bool ok_slot = ok_h[h];
    const CS mfg_action& ac = S->s.actions[al][ok_slot ? my_act[h] : 0];
    const int op = ok_slot ? ac.op : -1;
    const int pos = pos_h[h];
    const bool act = me && al0 < F && !par;
    // DoorUse: the present doors in the 3x3 around the agent (doors/actions.py:18-34)
    const int x = pos >= 0 ? pos / W : 0, y = pos >= 0 ? pos - x * W : 0;
    u64 tm[NW];
#pragma unroll
    for (int g = 0; g < NW; g++) tm[g] = 0;
    if (act && op == MFG_ACT_DOORUSE) {
      for (int k = 0; k < 9; k++) {
        const int px = x + k / 3 - 1, py = y + k % 3 - 1;
        if (px < 0 || py < 0 || px >= S->s.H || py >= W) continue;
        const int c = px * W + py;
        if (S->level[c] == 1) continue;
        const int d = S->door_of[c];
        if (d != 0xFF && (e.door()[d] & DW_PRESENT)) mask_set(tm, d);
      }
    }
    const u64 tm_lanes = ballot(mask_any(tm));
    u64 seen[NW];  // doors toggled by DoorUse agents of this pass before this one
#pragma unroll
    for (int g = 0; g < NW; g++) seen[g] = 0;
    for (u64 m = tm_lanes; m; m &= m - 1) {
      const int b = ffs64(m);
#pragma unroll
      for (int g = 0; g < NW; g++) {
        const u64 tb = ((u64)(uint32_t)rl((int)(uint32_t)(tm[g] >> 32), b) << 32) | (uint32_t)rl((int)(uint32_t)tm[g], b);
        if (b < lane) seen[g] ^= tb;
      }
    }
    // Move: target, blocking as this agent sees it (walls, closed present doors; states.py:240-270)
    static const int DX[8] = {-1, -1, 0, 1, 1, 1, 0, -1};
    static const int DY[8] = {0, 1, 1, 1, 0, -1, -1, -1};
    const bool mv = act && op == MFG_ACT_MOVE;
    const int t = mv ? pos + DX[ac.arg] * W + DY[ac.arg] : 0;  // levels are wall-bounded
    bool blocked = false;
    if (mv) {
      blocked = S->level[t] == 1;
      const int d = S->door_of[t];
      if (!blocked && d != 0xFF) {
        const int w = e.door()[d];
        const bool open = ((w & DW_OPEN) != 0) ^ mask_get(seen, d);
        blocked = (w & DW_PRESENT) && !open;
      }
    }
    const bool vmove = mv && !blocked && t != pos;
    const int npos = vmove ? t : pos;
    // occupancy seen by this agent at X (its target, or its own cell for Charge)
    const int X = mv ? t : pos;
    int cnt = 0;
    const int na = min(A - h * MFG_WAVE, MFG_WAVE);
    for (int b = 0; b < na; b++) {
      const int nb = rl(npos, b), ob = rl(pos, b);
      cnt += (b < lane) ? (nb == X) : ((b > lane) ? (ob == X) : 0);
    }
    if constexpr (NW > 1) {  // the other passes' agents from the record: earlier passes committed, later ones not yet
      for (int b = 0; b < h * MFG_WAVE; b++) cnt += e.agpos()[b] == X;
      for (int b = (h + 1) * MFG_WAVE; b < A; b++) cnt += e.agpos()[b] == X;
    }
    int mcnt = 0;  // maintainers collide with a mover (colliders_at); Charge counts agents only
    const int nk = S->kmax ? e.H(H_N_MAINTS) : 0;
    for (int k = 0; k < nk; k++) { const int w = e.maints()[k]; mcnt += (EW_POS(w) == X && (w & EW_PRESENT)) ? 1 : 0; }
    int valid = 0, coll = 0;
    if (act) {
      if (op == MFG_ACT_NOOP) valid = 1;
      else if (op == MFG_ACT_MOVE) { valid = vmove; coll = vmove ? cnt + mcnt > 0 : 1; }
      else if (op == MFG_ACT_DOORUSE) valid = mask_any(tm);
      else if (op == MFG_ACT_CHARGE) {  // batteries/actions.py:20-31, entitites.py:98-111
        bool pod = false;
        const int np = e.H(H_N_PODS);
        for (int i = 0; i < np; i++) { const int w = e.pods()[i]; pod |= EW_POS(w) == pos && (w & EW_ALIVE); }
        const double ch = e.bat()[al];
        if (pod && ch < 1.0 && cnt == 0) {
          const double nv = S->s.pod_charge_rate + ch;
          e.bat()[al] = nv > 1.0 ? 1.0 : nv;
          valid = 1;
        }
      }  // ItemAction here: no item, no drop-off on the cell -> fails
    }
    // commit: positions + arrival order, doors, debt, rewards and events
    const u64 vm = ballot(vmove);
    const int arr0 = e.H(H_ARRIVAL);
    const int debt = popc(ballot(mv && !blocked)) + popc(vm);
    wave_sync();
    if (vmove) {
      e.agpos()[al] = t;
      e.agarr()[al] = arr0 + mbcnt(vm);
    }
    if (tm_lanes) {  // each door: the parity of its toggles; opening resets the timer
#pragma unroll
      for (int g = 0; g < NW; g++) {
        const int dl = g * MFG_WAVE + lane;
        if (dl >= S->nd) continue;
        int n = 0;
        for (u64 m = tm_lanes; m; m &= m - 1) {
          const int b = ffs64(m);
          const uint32_t lo = (uint32_t)rl((int)(uint32_t)tm[g], b), hi = (uint32_t)rl((int)(uint32_t)(tm[g] >> 32), b);
          n += ((lane < 32 ? lo : hi) >> (lane & 31)) & 1;
        }
        if (n) {
          const int w = e.door()[dl];
          const bool open0 = (w & DW_OPEN) != 0;
          const bool opened = open0 ? n >= 2 : true;
          const bool open = open0 ^ ((n & 1) != 0);
          e.door()[dl] = (w & DW_PRESENT) | (open ? DW_OPEN : 0) | ((opened ? (S->s.door_auto_close & 0xFF) : DW_TTC(w)) << 8);
        }
      }
    }
    if (lane == 0) {
      e.hdr()[H_ARRIVAL] = arr0 + popc(vm);
      e.hdr()[H_DEBT] += debt;
    }
    if (act) {
      o.my_rew[h] += valid ? ac.valid_reward : ac.fail_reward;
      o.my_act_ev[h] = 0x80 | (valid ? 1 : 0) | (coll ? 2 : 0);
      o.my_slot[h] = my_act[h];
    }
    wave_sync();
  }
  return F;
}

// ------------------------------------------------------------------------------------------------
// rules (environment/rules.py, modules/*/rules.py); hook order states.py:170-226
// ------------------------------------------------------------------------------------------------
// ------------------------------------------------------------------------------------------------
// maintainers (maintenance/entities.py:17-136, rules.py:9-40) and the floor graph (states.py:82-87)
// ------------------------------------------------------------------------------------------------
// one 32-bit MT19937 output (the floor-shuffle debt must be paid first: the stream is shared)
__device__ uint32_t mt_u32(const Env& e) {
  int idx = e.H(H_MT_IDX);
  if (idx >= 624) {
    mt_twist(e);
    idx = 0;
  }
  const uint32_t y = (uint32_t)uni((int)mt_temper(e.mt()[idx]));
  e.setH(H_MT_IDX, idx + 1);
  wave_sync();
  return y;
}
// random._randbelow_with_getrandbits(n) (random.py:239-249), n >= 1
__device__ int mt_randbelow1(const Env& e, int n) {
  const int k = 32 - __clz(n);
  int r = (int)(mt_u32(e) >> (32 - k));
  while (r >= n) r = (int)(mt_u32(e) >> (32 - k));
  return r;
}

#define BFS_ABSENT 0xFFFFu
#define BFS_ROOT 0xFFFEu
// neighbours of floor node f in adjacency order: points_to_graph (algorithms/static/utils.py:7-41) adds the
// edges of itertools.combinations(floorlist, 2) in order, so every adjacency lists its neighbours by
// ascending build-time rank. nb[k] = rank << 16 | floor index, sorted (a fixed 19-exchange network keeps
// everything in registers); missing neighbours sort last as 0xFFFFFFFF. Returns the neighbour count.
__device__ __forceinline__ void cx(uint32_t& a, uint32_t& b) {
  const uint32_t lo = min(a, b), hi = max(a, b);
  a = lo;
  b = hi;
}
__device__ __forceinline__ int graph_adj(const Env& e, int f, uint32_t (&nb)[8]) {
  SpecP S = e.S;
  const int W = S->s.W, c = S->floor_init[f], x = c / W, y = c % W;
  const uint16_t* rk = e.grank();
  int n = 0;
#pragma unroll
  for (int d = 0; d < 8; d++) {
    const int dx = d < 3 ? -1 : (d == 3 || d == 7 ? 0 : 1);
    const int dy = (d == 0 || d == 5) ? -1 : ((d == 1 || d == 6) ? 0 : (d == 3 ? -1 : 1));
    const int nx = x + dx, ny = y + dy;
    const bool in = nx >= 0 && ny >= 0 && nx < S->s.H && ny < W;
    const int g = in ? S->cell_f[nx * W + ny] : -1;
    nb[d] = g >= 0 ? ((uint32_t)rk[g] << 16) | (uint32_t)g : 0xFFFFFFFFu;
    n += g >= 0;
  }
  cx(nb[0], nb[1]); cx(nb[2], nb[3]); cx(nb[4], nb[5]); cx(nb[6], nb[7]);
  cx(nb[0], nb[2]); cx(nb[1], nb[3]); cx(nb[4], nb[6]); cx(nb[5], nb[7]);
  cx(nb[1], nb[2]); cx(nb[5], nb[6]); cx(nb[0], nb[4]); cx(nb[3], nb[7]);
  cx(nb[1], nb[5]); cx(nb[2], nb[6]);
  cx(nb[1], nb[4]); cx(nb[3], nb[6]);
  cx(nb[2], nb[4]); cx(nb[3], nb[5]);
  cx(nb[3], nb[4]);
  return n;
}
__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = min(v, (uint32_t)__shfl_xor((int)v, o));
  return v;
}
// exclusive prefix sum over lanes
__device__ __forceinline__ int wave_excl_scan(int v, int lane) {
  int x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(x, o);
    if (lane >= o) x += y;
  }
  return x - v;
}
// BFS scratch may live in HBM (e.bfs in the per-env pool): lanes exchange through it after a
// workgroup-scope fence (s_waitcnt on both LDS and vector memory), not just the wave barrier
__device__ __forceinline__ void bfs_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
  __builtin_amdgcn_wave_barrier();
}
// nx.shortest_path(floortile_graph, src, dst) == nx.bidirectional_shortest_path: networkx 3.4.2
// _bidirectional_pred_succ restated level-synchronously and exactly. The sequential search visits the
// candidates (fringe index i, adjacency slot k) of a level in (i, k) order; here every lane expands fringe
// nodes and the order is recovered from keys i*8+k: the meeting point is the smallest key whose neighbour
// is in the other tree, a node's parent is its smallest discovering key (LDS atomicMin), and the new fringe
// is the discoveries compacted in key order. Route (floor indices) into `route`, returns its length or -1
// (NodeNotFound / NetworkXNoPath / longer than cap: a crash upstream, or engine capacity).
__device__ int bfs_route(const Env& e, int src, int dst, uint16_t* route, int cap) {
  SpecP S = e.S;
  const int nf = S->nf, lane = e.lane;
  if (!S->node_ok[src] || !S->node_ok[dst]) return -1;
  if (src == dst) {
    if (lane == 0) route[0] = (uint16_t)src;
    bfs_sync();
    return 1;
  }
  uint16_t* pred = (uint16_t*)e.bfs;
  uint16_t* succ = pred + nf;
  uint16_t* ff = succ + nf;
  uint16_t* rf = ff + nf;
  uint16_t* lvl = rf + nf;
  uint32_t* disc = (uint32_t*)(((uintptr_t)(lvl + nf) + 3) & ~(uintptr_t)3);
  for (int i = lane; i < nf; i += MFG_WAVE) { pred[i] = BFS_ABSENT; succ[i] = BFS_ABSENT; disc[i] = 0xFFFFFFFFu; }
  bfs_sync();
  if (lane == 0) { pred[src] = BFS_ROOT; succ[dst] = BFS_ROOT; ff[0] = (uint16_t)src; rf[0] = (uint16_t)dst; }
  bfs_sync();
  int nff = 1, nrf = 1, meet = -1, level = 0;
  while (nff && nrf && meet < 0) {
    const bool fwd = nff <= nrf;
    uint16_t* F = fwd ? ff : rf;
    uint16_t* mine = fwd ? pred : succ;
    const uint16_t* other = fwd ? succ : pred;
    const int n = fwd ? nff : nrf;
    for (int i = lane; i < n; i += MFG_WAVE) lvl[i] = F[i];
    bfs_sync();
    const uint32_t tag = (uint32_t)(4095 - (level & 4095)) << 20;  // newer levels win atomicMin
    level++;
    // pass 1: the meeting candidate
    uint32_t mk = 0xFFFFFFFFu;
    for (int b = 0; b < n; b += MFG_WAVE) {
      const int i = b + lane;
      uint32_t nb[8];
      const int m = graph_adj(e, lvl[i < n ? i : 0], nb);
#pragma unroll
      for (int k = 0; k < 8; k++)
        if (i < n && k < m && other[nb[k] & 0xFFFFu] != BFS_ABSENT) mk = min(mk, (uint32_t)(i * 8 + k));
    }
    mk = wave_min_u32(mk);
    // pass 2: discoveries up to and including the meeting candidate
    for (int b = 0; b < n; b += MFG_WAVE) {
      const int i = b + lane;
      uint32_t nb[8];
      const int m = graph_adj(e, lvl[i < n ? i : 0], nb);
#pragma unroll
      for (int k = 0; k < 8; k++) {
        const uint32_t key = (uint32_t)(i * 8 + k), g = nb[k] & 0xFFFFu;
        if (i < n && k < m && key <= mk && mine[g] == BFS_ABSENT) atomicMin(&disc[g], tag | key);
      }
    }
    bfs_sync();
    // pass 3: commit parents; the new fringe in key order
    int cnt_total = 0;
    for (int b = 0; b < n; b += MFG_WAVE) {
      const int i = b + lane;
      uint32_t nb[8];
      const int m = graph_adj(e, lvl[i < n ? i : 0], nb);
      const int vi = i < n ? (int)lvl[i] : 0;
      uint32_t win = 0;
#pragma unroll
      for (int k = 0; k < 8; k++) {
        const uint32_t key = (uint32_t)(i * 8 + k);
        if (i < n && k < m && key <= mk && disc[nb[k] & 0xFFFFu] == (tag | key)) win |= 1u << k;
      }
      const int cnt = __popc(win);
      const int off = cnt_total + wave_excl_scan(cnt, lane);
      int q = 0;
#pragma unroll
      for (int k = 0; k < 8; k++) {
        if ((win >> k) & 1u) {
          mine[nb[k] & 0xFFFFu] = (uint16_t)vi;
          F[off + q] = (uint16_t)(nb[k] & 0xFFFFu);
          q++;
        }
      }
      cnt_total = __shfl(off + cnt, 63);  // off already includes the earlier passes
    }
    bfs_sync();
    if (mk != 0xFFFFFFFFu) {
      // the meeting node: neighbour mk & 7 of fringe node mk >> 3
      uint32_t nb[8];
      graph_adj(e, lvl[mk >> 3], nb);
      uint32_t g = 0;
#pragma unroll
      for (int k = 0; k < 8; k++)
        if ((int)(mk & 7u) == k) g = nb[k] & 0xFFFFu;
      meet = uni((int)g);
    } else if (fwd) {
      nff = cnt_total;
    } else {
      nrf = cnt_total;
    }
  }
  if (meet < 0) return -1;
  // path: meet -> pred chain to src (reversed), then the succ chain to dst (lane 0, sequential)
  int len = 0;
  if (lane == 0) {
    int n = 0;
    for (int w = meet; w != BFS_ROOT && n <= cap; w = pred[w]) n++;
    int m = 0;
    for (int w = succ[meet]; w != BFS_ROOT && n + m <= cap; w = succ[w]) m++;
    len = n + m;
    if (len <= cap) {
      int k = n - 1;
      for (int w = meet; w != BFS_ROOT; w = pred[w]) route[k--] = (uint16_t)w;
      k = n;
      for (int w = succ[meet]; w != BFS_ROOT; w = succ[w]) route[k++] = (uint16_t)w;
    } else {
      len = -1;
    }
  }
  len = rl(len, 0);
  bfs_sync();
  return len;
}
// Maintainer.calculate_route: route[1:] as cells into the maintainer's path; false on failure
__device__ bool maint_route(const Env& e, int k, int target_cell, int* crashed) {
  SpecP S = e.S;
  int* st = e.mst(k);
  const int pos = EW_POS(uni(e.maints()[k]));
  uint16_t* route = (uint16_t*)e.scratch;  // scratch_bytes >= 2 * (path_cap + 2)
  if (!e.H(H_GRAPH_BUILT)) {  // Gamestate.floortile_graph: points_to_graph(self.entities.floorlist), once
    pay_debt(e);
    floor_shuffle(e);
    for (int i = e.lane; i < S->nf; i += MFG_WAVE) e.grank()[S->cell_f[e.perm()[i]]] = (uint16_t)i;
    e.setH(H_GRAPH_BUILT, 1);
    wave_sync();
  }
  const int n = bfs_route(e, S->cell_f[pos], S->cell_f[target_cell], route, S->path_cap + 1);
  if (n < 0) { *crashed = 2; return false; }  // NodeNotFound / NetworkXNoPath (or route > path_cap)
  uint16_t* path = e.mpath(k);
  for (int i = e.lane; i < n - 1; i += MFG_WAVE) path[i] = (uint16_t)S->floor_init[route[i + 1]];
  wave_sync();
  if (e.lane == 0) { st[MS_PATH_N] = n - 1; st[MS_PATH_HEAD] = 0; }
  wave_sync();
  return true;
}
// Entity.move of maintainer k to `cell` (entity.py:175-199): global pos_dict by identifier (Q14)
__device__ void maint_move(const Env& e, int k, int cell) {
  const int id = e.H(H_MAINT_BASE) + k;
  const int old = EW_POS(uni(e.maints()[k]));
  global_remove_id(e, old, id);
  int slot;
  const bool present = find_present_id(e, cell, id, &slot) == K_NONE;
  wave_sync();
  if (e.lane == 0) e.maints()[k] = cell | EW_ALIVE | (present ? EW_PRESENT : 0);
  wave_sync();
}
// Maintainer.tick (maintenance/entities.py:37-62); MoveMaintainers discards every result
template <int NW>
__device__ void maint_tick(const Env& e, int k, int* crashed) {
  SpecP S = e.S;
  const int W = S->s.W;
  int* st = e.mst(k);
  const int pos = EW_POS(uni(e.maints()[k]));
  const int nM = e.H(H_N_MACHINES);
  const u64 mm = grp_at(e.machines(), nM, pos, EW_ALIVE, e.lane);
  if (mm) {
    const int mid = e.H(H_MACHINE_BASE) + ffs64(mm);
    if (mid != uni(st[MS_LAST_SERVICED])) {
      // MachineAction.do -> Machine.maintain(): idle with health 100 > 98, not valid, no change (Q18)
      wave_sync();
      if (e.lane == 0) st[MS_LAST_SERVICED] = mid;
      wave_sync();
      return;
    }
  }
  // get_move_action (:64-103)
  if (uni(st[MS_PATH_HEAD]) >= uni(st[MS_PATH_N])) {
    int nn = uni(st[MS_NEXT_N]);
    if (!nn) {
      pay_debt(e);
      if (free_positions(e, 1, e.scratch) < 1) { *crashed = 3; return; }  // random_free_position
      const int fp = uni(e.scratch[0]);
      int* nx = st + MS_NEXT;
      if (e.lane == 0) {
        for (int i = 0; i < nM; i++) nx[i] = EW_POS(e.machines()[i]);
        nx[nM] = fp;
      }
      nn = nM + 1;
      wave_sync();
      for (int i = nn - 1; i > 0; i--) {  // shuffle(self._next) (random.py:380-395)
        const int j = mt_randbelow1(e, i + 1);
        if (e.lane == 0) { const int t = nx[i]; nx[i] = nx[j]; nx[j] = t; }
        wave_sync();
      }
    }
    int t = uni(st[MS_NEXT + nn - 1]);
    nn--;
    if (!maint_route(e, k, t, crashed)) return;
    if (uni(st[MS_PATH_N]) == 0) {
      if (!nn) { *crashed = 4; return; }  // pop from an empty list
      t = uni(st[MS_NEXT + nn - 1]);
      nn--;
      if (!maint_route(e, k, t, crashed)) return;
    }
    wave_sync();
    if (e.lane == 0) st[MS_NEXT_N] = nn;
    wave_sync();
  }
  const int head = uni(st[MS_PATH_HEAD]);
  if (head >= uni(st[MS_PATH_N])) { *crashed = 5; return; }  // self._path[0] on an empty path
  const int nxt = uni(e.mpath_at(k, head));
  const int d = door_idx(e, nxt);
  if (d >= 0 && !(e.door()[d] & DW_OPEN)) {  // _closed_door_in_path -> DoorUse
    door_use_at<NW>(e, pos / W, pos % W);
    return;
  }
  if (colliders_at<NW>(e, nxt) > 0) return;  // _predict_move: a collider ahead -> Noop
  wave_sync();
  if (e.lane == 0) st[MS_PATH_HEAD] = head + 1;
  wave_sync();
  const int dx = nxt / W - pos / W, dy = nxt % W - pos % W;
  if (dx < -1 || dx > 1 || dy < -1 || dy > 1 || (!dx && !dy)) { *crashed = 6; return; }  // not in MOVEMAP
  // Move.do (actions.py:77-100): check_move_validity, then Entity.move re-checks (Q3: one shuffle each)
  if (blocked_at<NW>(e, nxt)) return;
  int debt = 1;
  if (S->level[nxt] != 1) {
    debt++;
    maint_move(e, k, nxt);
  }
  e.setH(H_DEBT, e.H(H_DEBT) + debt);
  wave_sync();
}

template <bool RNG, bool MAINT, int NW>
__device__ void rule_tick_step(const Env& e, StepOut<NW>& o, int ri, int* scratch) {
  SpecP S = e.S;
  const CS mfg_rule& ru = S->s.rules[ri];
  const int op = ru.op;
  if (op == MFG_RULE_DOOR_AUTOCLOSE) {  // doors/rules.py:20-28, doors/entitites.py:107-122
    if (S->nd > 0) {
      const int nd = S->nd;
      int cnt[NW];
      door_cell_counts<NW>(e, e.scratch, false, cnt);  // per door lane: len(pos_dict[door])
      wave_sync();
#pragma unroll
      for (int g = 0; g < NW; g++) {
        const int d = g * MFG_WAVE + e.lane;
        if (d < nd) {
          int w = e.door()[d];
          if (cnt[g] <= 2) {
            const int ttc = DW_TTC(w);
            if ((w & DW_OPEN) && ttc) w = (w & ~0xFF00) | ((ttc - 1) << 8);
            else if ((w & DW_OPEN) && !ttc) w &= ~DW_OPEN;
          } else {
            w = (w & ~0xFF00) | ((S->s.door_auto_close & 0xFF) << 8);
          }
          e.door()[d] = w;
        }
      }
      wave_sync();
      o.door_autoclose = 1;
    }
  } else if (op == MFG_RULE_RESPAWN_ITEMS) {  // items/rules.py:28-33
    int c = uni(e.rctr()[ri]);
    if (!c) {
      if (S->s.items_quantity - e.H(H_N_ITEMS) > 0) o.crashed = 1;  // Item(pos, n, freq) TypeError upstream
    } else {
      wave_sync();
      if (e.lane == 0) e.rctr()[ri] = c - 1 > 0 ? c - 1 : 0;
      wave_sync();
    }
  } else if (op == MFG_RULE_BATTERY_DECHARGE || op == MFG_RULE_DONE_BATTERY) {  // batteries/rules.py:50-64
    bool missing = false;
#pragma unroll
    for (int h = 0; h < NW; h++) {
      const int a = h * MFG_WAVE + e.lane;
      if (a < S->A) {
        double cost = ru.f[0];
        if (ru.i[2])  // per_action_costs[agent.state.identifier]: the executed action's class, 'Noop' if paralyzed
          cost = o.my_slot[h] >= 0 ? S->s.actions[a][o.my_slot[h]].battery_cost : (ru.i[3] ? ru.f[3] : __builtin_nan(""));
        missing |= cost != cost;
        double b = e.bat()[a];
        if (b != 0.0 && cost == cost) {
          double nv = cost + b;
          e.bat()[a] = nv > 0.0 ? nv : 0.0;
        }
      }
    }
    if (ballot(missing)) o.crashed = MFG_CRASH_RULE;  // KeyError upstream
    wave_sync();
  } else if (op == MFG_RULE_RESPAWN_DIRT) {  // clean_up/rules.py:49-59
    int c = uni(e.rctr()[ri]);
    if (c < 0) {
    } else if (!c) {
      int valid = 0, v = 0;
      if constexpr (RNG) v = dirt_trigger_spawn(e, ru.i[1], ru.f[0], &valid, scratch);
      else o.crashed = 1;  // unreachable: the host stages the full record for specs with RespawnDirt
      o.dirt_spawn_value = v;
      o.dirt_spawn_valid = valid;
      wave_sync();
      if (e.lane == 0) e.rctr()[ri] = ru.i[0];
      wave_sync();
    } else {
      wave_sync();
      if (e.lane == 0) e.rctr()[ri] = c - 1;
      wave_sync();
    }
  } else if (op == MFG_RULE_MOVE_MAINTAINERS) {  // maintenance/rules.py:16-21
    if constexpr (RNG && MAINT) {
      const int nk = e.H(H_N_MAINTS);
      for (int k = 0; k < nk && !o.crashed; k++) maint_tick<NW>(e, k, &o.crashed);
    } else {
      o.crashed = 1;  // unreachable: the host launches k_logic<true, true> for specs with MoveMaintainers
    }
  } else if (op == MFG_RULE_DEST_REACH || op == MFG_RULE_DONE_DEST) {  // destinations/rules.py:34-54
    const int n = e.H(H_N_DESTS);
    for (int i = 0; i < n; i++) {
      const int w = uni(e.dests()[i]);
      if (w & EW_REACHED) continue;
      const int cell = EW_POS(w);
      // the agents on the cell; the Agents-group cell list is in arrival order, so the loop variable ends on the
      // last arrival
      int best = -1;
#pragma unroll
      for (int h = 0; h < NW; h++) {
        const int a = h * MFG_WAVE + e.lane;
        const bool on = a < S->A && e.agpos()[a < S->A ? a : 0] == cell;
        best = max(best, on ? e.agarr()[a] : -1);
      }
      for (int o2 = 32; o2 > 0; o2 >>= 1) best = max(best, __shfl_xor(best, o2));
      if (best < 0) continue;  // no agent there
      const int bnd = EW_BOUND(w);  // a bound destination is reached only by its agent (rules.py:40-46)
      if (bnd >= 0 && uni(e.agpos()[bnd]) != cell) continue;
      int last = -1;
#pragma unroll
      for (int h = NW - 1; h >= 0; h--) {
        const int a = h * MFG_WAVE + e.lane;
        const u64 lm = ballot(a < S->A && e.agpos()[a < S->A ? a : 0] == cell && e.agarr()[a < S->A ? a : 0] == best);
        if (lm) last = h * MFG_WAVE + ffs64(lm);
      }
      wave_sync();
      if (e.lane == 0) e.dests()[i] = w | EW_REACHED;
      wave_sync();
      agent_add(o.my_rew, last, e.lane, (double)ru.f[0]);
      // info: one '<agent>_<rule>' entry per credited destination; count per agent in ev_watch bits 3..7
#pragma unroll
      for (int h = 0; h < NW; h++)
        if (e.lane + h * MFG_WAVE == last) {
          if (o.my_watch_ev[h] >= (31 << 3)) e.hdr()[H_OVERFLOW] = 1;
          else o.my_watch_ev[h] += 1 << 3;
        }
      o.dest_reached++;
    }
  }
}

template <int NW>
__device__ void rule_post_step(const Env& e, StepOut<NW>& o, int ri) {
  SpecP S = e.S;
  const CS mfg_rule& ru = S->s.rules[ri];
  const int op = ru.op;
  if (op == MFG_RULE_RESPAWN_ITEMS) {  // items/rules.py:35-43
    int c = uni(e.rctr()[ri]);
    if (!c) {
      if (S->s.items_quantity - e.H(H_N_ITEMS) > 0) { o.crashed = 1; return; }
      o.respawn_items_value = S->s.items_quantity;
    } else {
      wave_sync();
      if (e.lane == 0) e.rctr()[ri] = c - 1 > 0 ? c - 1 : 0;
      wave_sync();
    }
  } else if (op == MFG_RULE_WATCH_COLLISIONS) {  // rules.py:276-307
    // Cells with >= 2 colliders (agents, closed doors, maintainers; walls never share a cell). Every collider
    // there gets one result unless an identifier-equal entity already got one this step. Only int
    // identifiers can clash (door index vs maintainer u_int), and door cells precede every other floor cell
    // in the pos_dict key order (walls and doors are keyed first at reset), so door cells are visited first
    // in door order; the order among the other cells cannot matter.
    const int A = S->A;
    const int nk = S->kmax ? e.H(H_N_MAINTS) : 0, mbase = S->kmax ? e.H(H_MAINT_BASE) : 0;
    bool hit = false;
    u64 used[NW];          // int identifiers < 64 NW that already have a result (door indices, maintainer ids)
    bool agres[NW];        // per agent: it has a result
#pragma unroll
    for (int h = 0; h < NW; h++) { used[h] = 0; agres[h] = false; }
    u64 mres = 0;          // maintainers with a result
    auto maint_results = [&](int cell) {
      const u64 mk = maints_at(e, cell);
      for (u64 m = mk; m; m &= m - 1) {
        const int k = ffs64(m), id = mbase + k;
        if ((mres >> k) & 1) continue;
        if (id < MFG_WAVE * NW && mask_get(used, id)) continue;
        mres |= 1ull << k;
        if (id < MFG_WAVE * NW) mask_set(used, id);
      }
    };
    // candidate cells first, lane-parallel (lane = door, then lane = agent); the ordered passes below
    // visit only cells with >= 2 colliders (usually none)
    const int nd = S->nd;
    int dcnt[NW];
    if (nd) door_cell_counts<NW>(e, e.scratch, true, dcnt);  // whole wave: every lane adds its entities
    u64 dcand[NW], acand[NW];
    int myp[NW];
#pragma unroll
    for (int g = 0; g < NW; g++) {
      dcand[g] = nd ? ballot(g * MFG_WAVE + e.lane < nd && dcnt[g] >= 2) : 0ull;
      const int a = g * MFG_WAVE + e.lane;
      myp[g] = a < A ? e.agpos()[a] : -1;
    }
    // agents on non-door cells: the other agents on the same cell (readlane loop) + maintainers there
    const int nkm = S->kmax ? e.H(H_N_MAINTS) : 0;
#pragma unroll
    for (int h = 0; h < NW; h++) {
      int na = 0;
#pragma unroll
      for (int g = 0; g < NW; g++) {
        const int ng = min(A - g * MFG_WAVE, MFG_WAVE);
        for (int b = 0; b < ng; b++) na += (rl(myp[g], b) == myp[h]) ? 1 : 0;
      }
      for (int k = 0; k < nkm; k++) { const int w = e.maints()[k]; na += (EW_POS(w) == myp[h] && (w & EW_PRESENT)) ? 1 : 0; }
      acand[h] = ballot(h * MFG_WAVE + e.lane < A && door_idx(e, myp[h] < 0 ? 0 : myp[h]) < 0 && na >= 2);
    }
#pragma unroll
    for (int g = 0; g < NW; g++)
      for (u64 dm = dcand[g]; dm; dm &= dm - 1) {
        const int d = g * MFG_WAVE + ffs64(dm);
        const int cell = S->door_cells[d];
        hit = true;
        if (present_closed_door(e, cell) && !mask_get(used, d)) { mask_set(o.door_coll, d); mask_set(used, d); }
#pragma unroll
        for (int h = 0; h < NW; h++)
          if (h * MFG_WAVE + e.lane < A && myp[h] == cell) agres[h] = true;
        maint_results(cell);
      }
#pragma unroll
    for (int h = 0; h < NW; h++)
      for (u64 am = acand[h]; am; am &= am - 1) {
        const int l = ffs64(am);
        const int cell = uni(e.agpos()[h * MFG_WAVE + l]);
        hit = true;
        if (e.lane == l) agres[h] = true;
        maint_results(cell);
      }
    for (int k = 0; k < nk; k++) {
      const int w = uni(e.maints()[k]);
      if (!(w & EW_PRESENT)) continue;
      const int cell = EW_POS(w);
      if (door_idx(e, cell) >= 0 || colliders_at<NW>(e, cell) < 2) continue;
      hit = true;
      maint_results(cell);
    }
#pragma unroll
    for (int h = 0; h < NW; h++)
      if (agres[h]) {
        if (!(o.my_watch_ev[h] & 1)) o.my_rew[h] += ru.f[0];
        o.my_watch_ev[h] |= 1;
      }
    o.maint_coll |= mres;
    if (ru.i[0] && hit) o.done_mask |= (int)(1u << 31);  // curr_done -> on_check_done
  } else if (op == MFG_RULE_BATTERY_DECHARGE || op == MFG_RULE_DONE_BATTERY) {  // batteries/rules.py:66-87
#pragma unroll
    for (int h = 0; h < NW; h++) {
      const int a = h * MFG_WAVE + e.lane;
      if (a < S->A) {
        const bool dis = e.bat()[a] == 0.0;
        int par = e.agpar()[a];
        if (dis) {
          o.my_rew[h] += ru.f[1];
          o.my_watch_ev[h] |= 2;
          if (ru.i[0]) par |= 1 << ri;
        }
        if (par && !dis) par &= ~(1 << ri);
        e.agpar()[a] = par;
      }
    }
    wave_sync();
  }
}

template <int NW>
__device__ void rule_check_done(const Env& e, StepOut<NW>& o, int ri) {
  SpecP S = e.S;
  const CS mfg_rule& ru = S->s.rules[ri];
  const int op = ru.op;
  if (op == MFG_RULE_DONE_MAXSTEPS) {
    if (ru.i[0] <= e.H(H_STEP)) { o.done = 1; o.done_mask |= 1 << ri; }
  } else if (op == MFG_RULE_WATCH_COLLISIONS) {
    if (ru.i[0] && (o.done_mask & (int)(1u << 31))) { o.done = 1; o.g_rew += ru.f[1]; }
  } else if (op == MFG_RULE_DONE_BATTERY) {  // batteries/rules.py:122-128
    int nz = 0;
#pragma unroll
    for (int h = 0; h < NW; h++) {
      const int a = h * MFG_WAVE + e.lane;
      nz += popc(ballot(a < S->A && e.bat()[a < S->A ? a : 0] == 0.0));
    }
    const bool any = nz != 0;
    const bool all = nz == S->A;
    if (ru.i[1] && (any || all)) { o.done = 1; o.done_mask |= 1 << ri; o.g_rew += ru.f[2]; }
  } else if (op == MFG_RULE_DONE_MAINT_COLLISION) {  // maintenance/rules.py:32-40
    const int nk = S->kmax ? e.H(H_N_MAINTS) : 0;
    bool any = false;
#pragma unroll
    for (int h = 0; h < NW; h++) {
      const int a = h * MFG_WAVE + e.lane;
      bool on = false;
      if (a < S->A) {
        const int p = e.agpos()[a];
        for (int k = 0; k < nk; k++) on |= EW_POS(e.maints()[k]) == p;
      }
      if (on) { o.my_rew[h] += ru.f[0]; o.my_watch_ev[h] |= 4; }
      any |= ballot(on) != 0;
    }
    if (any) { o.done = 1; o.done_mask |= 1 << ri; }
  } else if (op == MFG_RULE_DONE_DIRT) {  // clean_up/rules.py:22-25
    if (e.H(H_N_DIRT) == 0 && e.H(H_STEP)) { o.done = 1; o.done_mask |= 1 << ri; o.g_rew += ru.f[0]; }
  } else if (op == MFG_RULE_DONE_DEST) {  // destinations/rules.py:73-92
    const int n = e.H(H_N_DESTS);
    const bool rr = e.lane < n && (e.dests()[e.lane < n ? e.lane : 0] & EW_REACHED);
    const u64 m = ballot(rr);
    const bool any = m != 0, all = popc(m) == n;
    const int cond = ru.i[0];
    if ((cond == MFG_DEST_ANY && any) || (cond != MFG_DEST_ANY && all)) {
      o.done = 1; o.done_mask |= 1 << ri; o.g_rew += ru.f[1];
    } else if (cond == MFG_DEST_SIMULTANEOUS) {
      wave_sync();
      if (e.lane < n) e.dests()[e.lane] &= ~EW_REACHED;
      wave_sync();
    }
  }
}

// ------------------------------------------------------------------------------------------------
// reset (factory.py:134-148; global_entities.py:196-203; rules.py:182-199; SpawnEntity rules)
// ------------------------------------------------------------------------------------------------
template <int NW>
__device__ __attribute__((always_inline)) void env_reset(const Env& e, int* scratch) {
  SpecP S = e.S;
  const int A = S->A, W = S->s.W;
  int reset_crash = 0;  // a reference exception inside reset(): reported by the next step (crashed + done)
  pay_debt(e);
  // OBSBuilder keeps the episode-1 agent / battery objects for its ray origins and bound layers
  if (e.H(H_OBS_INIT) && !e.H(H_FROZEN)) {
#pragma unroll
    for (int h = 0; h < NW; h++) {
      const int a = h * MFG_WAVE + e.lane;
      if (a < A) {
        e.forg()[a] = e.agpos()[a];
        e.fgp()[a] = e.agpos()[a];
        e.fbat()[a] = e.bat()[a];
      }
    }
    e.setH(H_FROZEN, 1);
  }
  e.setH(H_STEP, 0);
  e.setH(H_CRASHED, 0);
  e.setH(H_N_ITEMS, 0); e.setH(H_N_PODS, 0); e.setH(H_N_DROPS, 0); e.setH(H_N_DIRT, 0); e.setH(H_N_DESTS, 0);
  e.setH(H_N_MACHINES, 0); e.setH(H_N_MAINTS, 0);
  for (int k = 0; k < S->kmax; k++) {  // maintainers are re-created: no path, no targets, 'None' serviced
    if (e.lane == 0) {
      e.mst(k)[MS_PATH_N] = 0; e.mst(k)[MS_PATH_HEAD] = 0; e.mst(k)[MS_NEXT_N] = 0; e.mst(k)[MS_LAST_SERVICED] = -1;
    }
  }
#pragma unroll
  for (int h = 0; h < NW; h++) {
    const int i = h * MFG_WAVE + e.lane;
    if (i < S->nd) e.door()[i] = DW_PRESENT | ((S->s.door_auto_close & 0xFF) << 8);  // closed
    if (i < A) { e.agpos()[i] = -1; e.agpar()[i] = 0; }
  }
  wave_sync();
  // SpawnAgents: per agent empty_positions (floor shuffle + filter + shuffle of the list) then pop().
  // At this point the only occupants of floor-list cells (every non-wall cell, doors included) are the doors,
  // all present after the reset, and the agents placed so far (each on its own non-door cell): a cell is empty
  // iff it is no door and no earlier agent stands on it, so empty_positions has nf - nd - a cells and the pick
  // scan tests the door table and the earlier agents' cells (lane b holds agent b's cell) instead of every
  // entity group per cell.
  int my_cell = -1;  // lane b < a: agent b's cell (agents 64.. are read from the record)
  for (int a = 0; a < A; a++) {
    floor_shuffle(e);
    const uint16_t* perm = e.perm();
    const int nf = S->nf;
    const int m = nf - S->nd - a;
    auto empty_at = [&](int cell) {
      bool occ = S->door_of[cell] != 0xFF;
      const int a0 = min(a, MFG_WAVE);
      for (int b = 0; b < a0; b++) occ |= rl(my_cell, b) == cell;
      if constexpr (NW > 1)
        for (int b = MFG_WAVE; b < a; b++) occ |= e.agpos()[b] == cell;
      return !occ;
    };
    // the draws of shuffle(empty_positions) on the replay's branch-free chunked path; the first accepted draw
    // (i = m - 1) picks the slot pop() takes
    const int j = m < 2 ? (m == 1 ? 0 : -1)
                        : (S->replay_top14 ? replay_shuffle_t<true, false>(e, nullptr, m - 1)
                                           : replay_shuffle_t<false, false>(e, nullptr, m - 1));
    int k = 0, cell = -1;
    const int npos = S->s.n_positions[a];
    if (npos > 0) {
      // configured Positions: get_first(x for x in positions if x in empty_positions) (rules.py:191-193, Q24),
      // then `assert state.check_pos_validity(position)`: one more floor shuffle (Q3); none -> ValueError
      for (int q = 0; q < npos && cell < 0; q++) {
        const int c = S->s.positions[a][q];
        if (S->level[c] != 1 && uni((int)empty_at(c))) cell = c;
      }
      if (cell >= 0) floor_shuffle(e);
      else reset_crash = MFG_CRASH_RULE;
    } else {
      for (int b = 0; b < nf && cell < 0; b += MFG_WAVE) {
        const int i = b + e.lane;
        const bool em = i < nf && empty_at(perm[i < nf ? i : 0]);
        const u64 mm = ballot(em);
        const int rank = k + mbcnt(mm);
        const u64 hitm = ballot(em && rank == j);
        if (hitm) cell = rl(i < nf ? (int)perm[i] : 0, ffs64(hitm));
        k += popc(mm);
      }
      if (cell < 0) reset_crash = MFG_CRASH_RULE;  // empty_positions.pop() on an empty list
    }
    if (cell < 0) cell = S->floor_init[0];
    wave_sync();
    if (e.lane == a) my_cell = cell;
    if (e.lane == 0) { e.agpos()[a] = cell; e.agarr()[a] = a; }
    e.setH(H_CNT_AGENT, e.H(H_CNT_AGENT) + 1);
    wave_sync();
  }
  e.setH(H_ARRIVAL, A);
  // rules' on_reset in order (states.py:45-50)
  for (int r = 0; r < S->s.n_rules; r++) {
    const CS mfg_rule& ru = S->s.rules[r];
    const int op = ru.op;
    if (op == MFG_RULE_SPAWN_BATTERIES) {
      e.setH(H_BAT_BASE, e.H(H_CNT_BATTERY));
      e.setH(H_CNT_BATTERY, e.H(H_CNT_BATTERY) + A);
#pragma unroll
      for (int h = 0; h < NW; h++)
        if (h * MFG_WAVE + e.lane < A) e.bat()[h * MFG_WAVE + e.lane] = S->s.battery_initial;
      wave_sync();
    } else if (op == MFG_RULE_SPAWN_PODS || op == MFG_RULE_SPAWN_DROPOFFS || op == MFG_RULE_SPAWN_ITEMS ||
               op == MFG_RULE_SPAWN_DESTS) {
      int hn, hb, hc;
      int* tbl;
      int q = ru.i[0];
      if (op == MFG_RULE_SPAWN_PODS) { hn = H_N_PODS; hb = H_POD_BASE; hc = H_CNT_POD; tbl = e.pods(); }
      else if (op == MFG_RULE_SPAWN_DROPOFFS) { hn = H_N_DROPS; hb = H_DROP_BASE; hc = H_CNT_DROP; tbl = e.drops(); }
      else if (op == MFG_RULE_SPAWN_DESTS) { hn = H_N_DESTS; hb = H_DEST_BASE; hc = H_CNT_DEST; tbl = e.dests(); }
      else { hn = H_N_ITEMS; hb = H_ITEM_BASE; hc = H_CNT_ITEM; tbl = e.items(); q -= e.H(H_N_ITEMS); }
      if (q > 0) {
        const int n = spawn_positions(e, q, ru.i[1], scratch);
        const int base = e.H(hc);
        e.setH(hb, base);
        for (int i = 0; i < n; i++) spawn_into(e, tbl, hn, base, scratch[i]);
        e.setH(hc, base + n);
        wave_sync();
      }
    } else if (op == MFG_RULE_SPAWN_DIRT) {
      int v;
      dirt_trigger_spawn(e, S->s.dirt_quantity, 0.0, &v, scratch);
    } else if (op == MFG_RULE_SPAWN_GLOBALPOS) {
      e.setH(H_CNT_GP, e.H(H_CNT_GP) + A);
    } else if (op == MFG_RULE_SPAWN_DEST_ON_AGENT) {  // destinations/rules.py:155-162: bound, on the agent's cell
      const int base = e.H(H_CNT_DEST);
      e.setH(H_DEST_BASE, base);
      for (int a = 0; a < A; a++) spawn_into(e, e.dests(), H_N_DESTS, base, uni(e.agpos()[a]), (a + 1) << EW_BOUND_SHIFT);
      e.setH(H_CNT_DEST, base + A);
      wave_sync();
    } else if (op == MFG_RULE_SPAWN_DEST_PER_AGENT) {  // destinations/rules.py:116-133
      const int base = e.H(H_CNT_DEST);
      e.setH(H_DEST_BASE, base);
      int made = 0;
      // candidate list after the 128 B of shuffle sink words at the start of the scratch
      uint16_t* l16 = (uint16_t*)((uint8_t*)scratch + 128);
      int* l32 = (int*)((uint8_t*)scratch + 128);
      for (int j = 0; j < S->s.n_dest_entries && !reset_crash; j++) {
        const int a = S->s.dest_entry_agent[j], apos = uni(e.agpos()[a]);
        const bool quant = S->s.dest_entry_q[j] > 0;
        int n;
        if (quant) {  // position_list = state.entities.floorlist (a shuffled copy), shuffled once more
          floor_shuffle(e);
          for (int i = e.lane; i < S->nf; i += MFG_WAVE) l16[i] = e.perm()[i];
          wave_sync();
          floor_shuffle_t(e, l16);
          n = S->nf;
        } else {      // coordinate list: shuffle(position_list) (random.py:380-395)
          n = S->s.dest_entry_n[j];
          if (e.lane < n) l32[e.lane] = S->s.dest_entry_cells[j][e.lane];
          wave_sync();
          for (int i = n - 1; i > 0; i--) {
            const int r2 = mt_randbelow1(e, i + 1);
            if (e.lane == 0) { const int t = l32[i]; l32[i] = l32[r2]; l32[r2] = t; }
            wave_sync();
          }
        }
        int cell = -1;  // pop() until a cell that is not the agent's and holds no destination; one per entry
        while (n > 0 && cell < 0) {
          const int c = quant ? (int)l16[n - 1] : uni(l32[n - 1]);
          n--;
          if (c != apos && !grp_at(e.dests(), e.H(H_N_DESTS), c, EW_ALIVE, e.lane)) cell = c;
        }
        if (cell < 0) { reset_crash = MFG_CRASH_RULE; break; }  // exit(-9999) upstream
        spawn_into(e, e.dests(), H_N_DESTS, base, cell, (a + 1) << EW_BOUND_SHIFT);
        made++;
      }
      e.setH(H_CNT_DEST, base + made);
      wave_sync();
    } else if (op == MFG_RULE_SPAWN_MACHINES || op == MFG_RULE_SPAWN_MAINTAINERS) {
      const bool mach = op == MFG_RULE_SPAWN_MACHINES;
      const int q = ru.i[0];
      const int n = spawn_positions(e, q, ru.i[1], scratch);
      const int hn = mach ? H_N_MACHINES : H_N_MAINTS, hc = mach ? H_CNT_MACHINE : H_CNT_MAINT;
      const int base = e.H(hc);
      e.setH(mach ? H_MACHINE_BASE : H_MAINT_BASE, base);
      for (int i = 0; i < n; i++) spawn_into(e, mach ? e.machines() : e.maints(), hn, base, scratch[i]);
      e.setH(hc, base + n);
      wave_sync();
    }
    wave_sync();
  }
  // rules' on_reset_post_spawn in order (states.py:52-56): DoRandomInitialSteps (rules.py:341-355)
  for (int r = 0; r < S->s.n_rules && !reset_crash; r++) {
    const CS mfg_rule& ru = S->s.rules[r];
    if (ru.op != MFG_RULE_RANDOM_INIT_STEPS) continue;
    for (int k = 0; k < ru.i[0] && !reset_crash; k++) {
      if (free_positions(e, 1, scratch) < 1) { reset_crash = MFG_CRASH_RULE; break; }  // random_free_position
      const int fp = uni(scratch[0]);
      const int fx = fp / W, fy = fp % W;
      // neighboring_4_positions: POS_MASK_4 offsets (helpers.py:34, not N/E/S/W: Q23) that are floor cells
      int* nb = scratch + 32;
      int n = 0;
      for (int q = 0; q < 6; q++) {
        const int dx = q == 1 || q == 3 ? -1 : (q == 2 || q == 5 ? 1 : 0), dy = q == 0 ? -1 : (q >= 3 ? 1 : 0);
        const int x = fx + dx, y = fy + dy;
        if (x >= 0 && y >= 0 && x < S->s.H && y < W && S->level[x * W + y] != 1) {
          if (e.lane == 0) nb[n] = x * W + y;
          n++;
        }
      }
      wave_sync();
      for (int i = n - 1; i > 0; i--) {  // random.shuffle(neighbor_positions)
        const int r2 = mt_randbelow1(e, i + 1);
        if (e.lane == 0) { const int t = nb[i]; nb[i] = nb[r2]; nb[r2] = t; }
        wave_sync();
      }
      const int p = n ? uni(nb[n - 1]) : -1;
      // get_first(by_pos(p)): the Agents group lists a cell's agents in arrival order
      int arr = 0x7FFFFFFF;
#pragma unroll
      for (int h = 0; h < NW; h++) {
        const int b = h * MFG_WAVE + e.lane;
        const bool on = p >= 0 && b < A && e.agpos()[b < A ? b : 0] == p;
        arr = min(arr, on ? e.agarr()[b] : 0x7FFFFFFF);
      }
      for (int o2 = 32; o2 > 0; o2 >>= 1) arr = min(arr, __shfl_xor(arr, o2));
      if (arr == 0x7FFFFFFF) { reset_crash = MFG_CRASH_RULE; break; }  // pop() on an empty list / assert isinstance
      int a = -1;
#pragma unroll
      for (int h = NW - 1; h >= 0; h--) {
        const int b = h * MFG_WAVE + e.lane;
        const u64 am = ballot(b < A && e.agpos()[b < A ? b : 0] == p && e.agarr()[b < A ? b : 0] == arr);
        if (am) a = h * MFG_WAVE + ffs64(am);
      }
      // chosen_agent.move(free_pos) (entity.py:175-199): check_move_validity once (states.py:240-270, Q3)
      const bool blocked = blocked_at<NW>(e, fp);
      if (!blocked) floor_shuffle(e);
      const bool not_blocked = !blocked && S->level[fp] != 1;
      const bool blocking_others = S->s.agent_blocking[a] && (colliders_at<NW>(e, fp) > 0 || blocked);
      if (p != fp && not_blocked && !blocking_others) set_agent_pos(e, a, fp);
    }
  }
  if (reset_crash) e.setH(H_CRASHED, reset_crash);
  e.setH(H_EPISODE, e.H(H_EPISODE) + 1);
  wave_sync();
}

// ------------------------------------------------------------------------------------------------
// observation (observation_builder.py:138-235, ray_caster.py:66-104)
// ------------------------------------------------------------------------------------------------
// Per-env cell map (one byte per grid cell, in LDS), built once per render and shared by all agents:
// walls come from the static base map, the dynamic entities are OR-ed in. The ray walk reads its
// light blockers from it and the placement reads each window cell's tag bits with one LDS load.
// Bits 0..6 sit at their obs tag's bit (MFG_TAG_*), machines/maintainers one above theirs, so the placement's
// tag word is a mask and a shift instead of one test per entity kind; the byte map (no machines or
// maintainers) uses bits 0..7.
#define CM_WALL 1u       // wall (static)
#define CM_DOOR 2u       // door present in the global pos_dict
#define CM_ITEM 4u
#define CM_POD 8u
#define CM_DROP 16u
#define CM_DIRT 32u
#define CM_DEST 64u      // destination present and not reached
#define CM_DCLOSED 128u  // door present and closed (blocks light, encodes 0.6666)
#define CM_MACHINE 256u
#define CM_MAINT 512u
static_assert(CM_WALL == 1u << MFG_TAG_WALLS && CM_DOOR == 1u << MFG_TAG_DOORS && CM_ITEM == 1u << MFG_TAG_ITEMS &&
                  CM_POD == 1u << MFG_TAG_PODS && CM_DROP == 1u << MFG_TAG_DROPOFFS && CM_DIRT == 1u << MFG_TAG_DIRT &&
                  CM_DEST == 1u << MFG_TAG_DESTS && CM_MACHINE == 2u << MFG_TAG_MACHINES &&
                  CM_MAINT == 2u << MFG_TAG_MAINTAINERS,
              "cell-map bits follow the obs tag bits");

__device__ __forceinline__ int v_clamp(int v, int n) { return v < 0 ? 0 : (v >= n ? n - 1 : v); }
template <bool MM>
__device__ __forceinline__ uint32_t cmap_at(const Env& e, int cell) {
  return MM ? (uint32_t)((const uint16_t*)e.cmap)[cell] : (uint32_t)e.cmap[cell];
}
template <bool MM>
__device__ __forceinline__ bool light_block(const Env& e, int x, int y) {
  SpecP S = e.S;
  if (x < 0 || y < 0 || x >= S->s.H || y >= S->s.W) return false;
  return (cmap_at<MM>(e, x * S->s.W + y) & (CM_WALL | CM_DCLOSED)) != 0;
}
// the same without branches: the cell index is clamped to 0 outside the grid, and the test masked
template <bool MM>
__device__ __forceinline__ bool light_block_bf(const Env& e, int x, int y) {
  SpecP S = e.S;
  const bool inb = ((unsigned)x < (unsigned)S->s.H) & ((unsigned)y < (unsigned)S->s.W);
  const uint32_t c = cmap_at<MM>(e, inb ? x * S->s.W + y : 0);
  return inb & ((c & (CM_WALL | CM_DCLOSED)) != 0);
}
template <bool MM>
__device__ __forceinline__ void cmap_or(const Env& e, int cell, uint32_t bit) {
  if (MM) atomicOr((uint32_t*)(e.cmap + 2 * (cell & ~1)), bit << (16 * (cell & 1)));
  else atomicOr((uint32_t*)(e.cmap + (cell & ~3)), bit << (8 * (cell & 3)));
}
// waves of one env's workgroup (multi-wave render): a workgroup barrier; single-wave: the wave barrier
template <bool MW>
__device__ __forceinline__ void mw_sync() {
  if constexpr (MW) __syncthreads();
  else wave_sync();
}
template <bool MM, bool MW = false>
__device__ void build_cmap(const Env& e, int wv = 0, int nwv = 1) {
  SpecP S = e.S;
  const int lane = e.lane;
  const int n16 = (MM ? S->map_bytes : S->map_bytes8) >> 4;
  const uint4* src = MM ? (const uint4*)S->base_map : (const uint4*)S->base_map8;
  for (int i = wv * MFG_WAVE + lane; i < n16; i += MFG_WAVE * nwv) ((uint4*)e.cmap)[i] = src[i];
  mw_sync<MW>();
  if (MW && wv) return;  // the dynamic entities: one wave (the others wait at the caller's barrier)
  for (int d = lane; d < S->nd; d += MFG_WAVE) {
    const int w = e.door()[d];
    if (w & DW_PRESENT) cmap_or<MM>(e, S->door_cells[d], CM_DOOR | ((w & DW_OPEN) ? 0u : CM_DCLOSED));
  }
  auto grp = [&](const int* tbl, int n, uint32_t bit, bool dest) {
    for (int i = lane; i < n; i += MFG_WAVE) {
      const int w = tbl[i];
      if ((w & EW_PRESENT) && EW_POS(w) != EW_NOPOS && !(dest && (w & EW_REACHED))) cmap_or<MM>(e, EW_POS(w), bit);
    }
  };
  grp(e.items(), e.H(H_N_ITEMS), CM_ITEM, false);
  grp(e.pods(), e.H(H_N_PODS), CM_POD, false);
  grp(e.drops(), e.H(H_N_DROPS), CM_DROP, false);
  grp(e.dests(), e.H(H_N_DESTS), CM_DEST, true);
  grp(e.dirtpos(), e.H(H_N_DIRT), CM_DIRT, false);
  if (MM && S->mmax) grp(e.machines(), e.H(H_N_MACHINES), CM_MACHINE, false);
  if (MM && S->kmax) grp(e.maints(), e.H(H_N_MAINTS), CM_MAINT, false);
  wave_sync();
}

// One ray per lane: packed (dx, dy) int8 offsets of up to MAXPTS points and the ray length. Point masks are 32-bit
// for rays of up to 32 points, 64-bit above (pomdp_r 16..31, full observability on levels with min(H, W) <= 63).
template <int MAXPTS>
struct RayLane {
  static_assert(MAXPTS <= 64, "rays of at most 64 points");
  typedef typename std::conditional<(MAXPTS > 32), u64, uint32_t>::type PM;  // one bit per point
  static constexpr int RSH = MAXPTS > 32 ? 6 : 5;  // first-visit rank = ray << RSH | point
  static constexpr int NW = (2 * MAXPTS + 3) / 4;
  uint32_t pk[NW];  // byte 2p = dx of point p, byte 2p+1 = dy (sign-extended on use)
  int len;
  PM diag;          // bit p: point p is a diagonal step
  __device__ __forceinline__ int dx(int p) const { return (int)(int8_t)((pk[p >> 1] >> ((p & 1) * 16)) & 0xFF); }
  __device__ __forceinline__ int dy(int p) const { return (int)(int8_t)((pk[p >> 1] >> ((p & 1) * 16 + 8)) & 0xFF); }
  static_assert(MAXPTS % 2 == 0 && NW * 4 == 2 * MAXPTS, "a ray's points are whole dwords");
  __device__ __forceinline__ void load(SpecP S, int ray) {
    const bool has = ray < S->nrays;
    // dword loads: a ray's 2 * MAXPTS bytes start on a 4-B boundary (MAXPTS is even, the table is a device
    // allocation)
    const uint32_t* pts = (const uint32_t*)S->ray_pts + (size_t)(has ? ray : 0) * NW;
#pragma unroll
    for (int q = 0; q < NW; q++) pk[q] = pts[q];
    len = has ? S->ray_len[ray] : 0;
    diag = has ? (PM)S->ray_diag[ray] : (PM)0;
  }
};

// Identifier-collision candidates (Q14), agent independent, built once per render into scratch:
// pair q = {cellA, cellB, codeA | codeB << 16}; code = kind << 12 | slot (kind: 1 door, 3 item, 4 pod,
// 5 drop, 6 dirt, 7 dest, 8 machine, 9 maintainer, 15 wall -> slot unused, the wall is identified by its
// cell). The dynamic int-id entities are the concatenation items, pods, drops, dests, dirt, machines,
// maintainers, handled 64 per pass. Returns the pair count (<= S->max_pairs, a bound from the group sizes).
// the first pairs_lds pairs live in LDS, the rest (rare: many colliding identifiers) in the env's HBM pool
// (explicit branches, not a pointer select, so LDS accesses stay ds_* instead of flat)
typedef __attribute__((address_space(3))) int lds_int;
typedef __attribute__((address_space(1))) int glb_int;
struct PairList {
  lds_int* lds;
  glb_int* glob;
  int nl;
  __device__ __forceinline__ void put(int q, int a, int b, int c) const {
    if (q < nl) { lds[3 * q] = a; lds[3 * q + 1] = b; lds[3 * q + 2] = c; }
    else { glb_int* g = glob + 3 * (q - nl); g[0] = a; g[1] = b; g[2] = c; }
  }
  __device__ __forceinline__ int get(int q, int k) const { return q < nl ? lds[3 * q + k] : glob[3 * (q - nl) + k]; }
  __device__ __forceinline__ void set(int q, int k, int v) const {
    if (q < nl) lds[3 * q + k] = v;
    else glob[3 * (q - nl) + k] = v;
  }
};
struct IdEnt {
  int kind, slot, cell, id;
};
template <bool MM>
__device__ __forceinline__ IdEnt id_entity(const Env& e, int l, int nI, int nP, int nR, int nS, int nT, int nM, int tot) {
  IdEnt r{0, 0, 0, -1};
  if (l >= tot) return r;
  int w;
  if (l < nI) { r.kind = K_ITEM; r.slot = l; w = e.items()[l]; r.id = e.hdr()[H_ITEM_BASE] + l; }
  else if ((l -= nI) < nP) { r.kind = K_POD; r.slot = l; w = e.pods()[l]; r.id = e.hdr()[H_POD_BASE] + l; }
  else if ((l -= nP) < nR) { r.kind = K_DROP; r.slot = l; w = e.drops()[l]; r.id = e.hdr()[H_DROP_BASE] + l; }
  else if ((l -= nR) < nS) { r.kind = K_DEST; r.slot = l; w = e.dests()[l]; r.id = e.hdr()[H_DEST_BASE] + l; }
  else if ((l -= nS) < nT) { r.kind = K_DIRT; r.slot = l; w = e.dirtpos()[l]; r.id = e.dirtid()[l]; }
  else if (!MM) { w = 0; }
  else if ((l -= nT) < nM) { r.kind = K_MACHINE; r.slot = l; w = e.machines()[l]; r.id = e.hdr()[H_MACHINE_BASE] + l; }
  else { l -= nM; r.kind = K_MAINT; r.slot = l; w = e.maints()[l]; r.id = e.hdr()[H_MAINT_BASE] + l; }
  if (!(w & EW_PRESENT)) r.id = -1;
  r.cell = EW_POS(w);
  return r;
}
template <bool MM>
__device__ int build_id_pairs(const Env& e, const PairList& pairs) {
  SpecP S = e.S;
  const int lane = e.lane, cap = S->max_pairs;
  const int nI = e.H(H_N_ITEMS), nP = e.H(H_N_PODS), nR = e.H(H_N_DROPS), nS = e.H(H_N_DESTS), nT = e.H(H_N_DIRT);
  const int nM = MM && S->mmax ? e.H(H_N_MACHINES) : 0, nK = MM && S->kmax ? e.H(H_N_MAINTS) : 0;
  const int tot = nI + nP + nR + nS + nT + nM + nK;
  int n = 0;
  auto emit = [&](bool has, int cA, int cB, int codes) {
    const u64 m = ballot(has);
    const int rank = n + mbcnt(m);
    if (has && rank < cap) pairs.put(rank, cA, cB, codes);
    n += popc(m);
  };
  for (int b = 0; b < tot; b += MFG_WAVE) {
    const IdEnt me = id_entity<MM>(e, b + lane, nI, nP, nR, nS, nT, nM, tot);
    const int code = (me.kind << 12) | me.slot;
    {  // wall partner Wall[id]
      const bool has = me.id >= 0 && me.id < S->nw;
      emit(has, me.cell, has ? S->wall_cells[me.id] : 0, code | (K_WALL << 28));
    }
    {  // door partner Door[id]
      const bool has = me.id >= 0 && me.id < S->nd && (e.door()[me.id < S->nd && me.id >= 0 ? me.id : 0] & DW_PRESENT);
      emit(has, me.cell, has ? S->door_cells[me.id] : 0, code | (((K_DOOR << 12) | me.id) << 16));
    }
    // dynamic-dynamic partners (different kinds, equal identifiers), oriented (earlier, later) in the
    // enumeration order items, pods, drop-offs, destinations, dirt, machines, maintainers. Every kind but dirt
    // numbers its identifiers base + slot, so the partner of kind k2 is slot id - base(k2): one lookup per
    // kind instead of a loop over all later entities. Non-dirt pairs are emitted from their earlier member,
    // dirt pairs from the dirt pile.
    const int mord = me.id < 0 ? -1 : (me.kind == K_ITEM ? 0 : me.kind == K_POD ? 1 : me.kind == K_DROP ? 2 :
                                       me.kind == K_DEST ? 3 : me.kind == K_DIRT ? 4 : me.kind == K_MACHINE ? 5 : 6);
    auto partner = [&](int k2, int o2, const int* tbl, int n2, int base2) {
      const int l2 = me.id - base2;
      const bool inr = mord >= 0 && o2 != mord && (unsigned)l2 < (unsigned)n2;
      const int w2 = tbl[inr ? l2 : 0];
      const bool later = o2 > mord;
      const bool has = inr && (w2 & EW_PRESENT) && (later || mord == 4);
      const int c2 = EW_POS(w2), code2 = (k2 << 12) | (inr ? l2 : 0);
      emit(has, later ? me.cell : c2, later ? c2 : me.cell, later ? (code | (code2 << 16)) : (code2 | (code << 16)));
    };
    if (nI) partner(K_ITEM, 0, e.items(), nI, e.H(H_ITEM_BASE));
    if (nP) partner(K_POD, 1, e.pods(), nP, e.H(H_POD_BASE));
    if (nR) partner(K_DROP, 2, e.drops(), nR, e.H(H_DROP_BASE));
    if (nS) partner(K_DEST, 3, e.dests(), nS, e.H(H_DEST_BASE));
    if (nM) partner(K_MACHINE, 5, e.machines(), nM, e.H(H_MACHINE_BASE));
    if (nK) partner(K_MAINT, 6, e.maints(), nK, e.H(H_MAINT_BASE));
  }
  // static Wall[k] / Door[k] pairs (host-filtered to pairs one ray fan can reach)
  for (int q0 = 0; q0 < S->n_wd_pairs; q0 += MFG_WAVE) {
    const int q = q0 + lane;
    bool has = q < S->n_wd_pairs;
    int k = 0, wc = 0, dc = 0;
    if (has) {
      k = S->wd_pairs[3 * q]; wc = S->wd_pairs[3 * q + 1]; dc = S->wd_pairs[3 * q + 2];
      has = (e.door()[k] & DW_PRESENT) != 0;
    }
    emit(has, dc, wc, ((K_DOOR << 12) | k) | (K_WALL << 28));
  }
  if (n > cap) e.setH(H_OVERFLOW, 1);
  mem_sync();
  return n < cap ? n : cap;
}

typedef __attribute__((address_space(3))) uint32_t lds_u32;
// the render's per-agent tables: LDS, or (long-ray render, k_obs_lr) the wave's HBM pool slot
template <bool LR>
using obs_u32 = typename std::conditional<LR, uint32_t, lds_u32>::type;
template <typename DP>
struct SupT {  // per-agent suppression sets from the identifier dedupe
  u64 items, pods, drops, dests, machines, maints;
  uint8_t* wsup;   // [dd] window cells whose wall or door is suppressed (both are static cells, one per cell; entities
                   // outside the window are never placed)
  DP* dsup;        // dirt slots: bitmap [dirt_cap / 32] (LDS; HBM in the long-ray render)
  int wx0, wy0, oh, ow, W;  // window origin cell and shape
  __device__ __forceinline__ bool dirt_sup(int i) const {
    return ((dsup[i >> 5] >> (i & 31)) & 1u) != 0;
  }
};
template <typename DP>
__device__ __forceinline__ void sup_add(SupT<DP>& s, int code, int xy, int lane) {
  const int kind = code >> 12, slot = code & 0xFFF;
  const u64 bit = 1ull << (slot & 63);
  switch (kind) {
    case K_ITEM: s.items |= bit; break;
    case K_POD: s.pods |= bit; break;
    case K_DROP: s.drops |= bit; break;
    case K_DEST: s.dests |= bit; break;
    case K_DIRT:
      if (lane == 0) s.dsup[slot >> 5] |= 1u << (slot & 31);
      break;
    case K_MACHINE: s.machines |= bit; break;
    case K_MAINT: s.maints |= bit; break;
    default: {  // a wall (K_WALL) or a door (K_DOOR): xy is its cell
      const int px = (xy >> 16) - s.wx0, py = (xy & 0xFFFF) - s.wy0;
      if (px >= 0 && py >= 0 && px < s.oh && py < s.ow && lane == 0) s.wsup[px * s.ow + py] = CM_WALL | CM_DOOR;
      break;
    }
  }
}

// packed obs rows + fused projection of one env (mfg_packed_obs, include/mfg.h), offset to this env
struct ObsPacked {
  uint16_t* idx;
  float* val;
  int* cnt;
  const float* wt;
  const float* bias;
  float* emb;
  int cap, E;
};

// MW: the env's workgroup has nwv waves (wave wv renders agents wv, wv + nwv, ...); they share the lean record,
// the cell map and the identifier pairs, each has its own per-agent tables after the shared part
// (S->lds_obs_shared + wv * S->lds_obs_wave)
#ifndef MFG_OBS_FLAT
// dense obs: the placement stashes each window cell's tags, visible agent mask and pile index, then writes the agent's
// [nl][dd] block as consecutive 64-value runs (lane = element) instead of one partial run per layer (0: per layer)
#define MFG_OBS_FLAT 1
#endif
#ifndef MFG_OBS_FLAT_MAXPTS
#define MFG_OBS_FLAT_MAXPTS 12  // renders with longer rays keep the per-layer stores (and no stashed tag table)
#endif
#ifndef MFG_OBS_FLAT_PK
#define MFG_OBS_FLAT_PK 1  // packed renders with wide windows queue their entries from the flattened pass too
#endif
#define CT_CLOSED 0x80000000u  // stashed tag word: the door on the cell is closed (tags stay below bit 16)
__device__ __forceinline__ uint32_t bperm(int src_lane, uint32_t v) {
  return (uint32_t)__builtin_amdgcn_ds_bpermute(src_lane << 2, (int)v);
}
// MAXPTS == 0 (LR): the long-ray render (rays of 65..255 points, k_obs_lr): each ray is walked in 32-point segments
// from the 16-bit ray table, and the per-agent tables (first-visit table, wall suppression, sinks, dirt bitmap,
// agent masks, dirt map, packed queue) live in the wave's HBM pool slot `slot` instead of LDS.
template <bool LR>
__device__ __forceinline__ void tbl_sync() {
  if constexpr (LR) {  // tables in HBM: stores and L2 atomics complete, and no stale L1 line is read afterwards
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "agent");
    __builtin_amdgcn_wave_barrier();
  } else {
    wave_sync();
  }
}
template <int MAXPTS, typename OT, bool MM, int PK, bool DIRT, bool MW>
__device__ void build_obs(const Env& e, OT* out_env, int* pair_glob, const ObsPacked& pk, int wv, int nwv,
                          int slot = 0) {
  SpecP S = e.S;
  constexpr bool LR = MAXPTS == 0;
  constexpr int RMP = LR ? 2 : MAXPTS;  // RayLane width (unused by the long-ray walk)
  typedef obs_u32<LR> tu32;
  // window: oh x ow cells from (wx0, wy0) = agent - r, or the whole level at (0, 0) when pomdp_r == 0
  // (observation_builder.py:152-158); rays and the first-visit table have radius fr (Q13)
  const int A = S->A, H = S->s.H, W = S->s.W, oh = S->oh, ow = S->ow, dd = S->dd, fr = S->fr;
  const bool full = S->r == 0;
  const float invw = 1.0f / (float)ow;
  const int lane = e.lane;
  const bool frozen = e.H(H_FROZEN) != 0;
  build_cmap<MM, MW>(e, wv, nwv);
  const PairList pairs{(lds_int*)e.scratch, (glb_int*)pair_glob, S->pairs_lds};
  int npairs = 0;
  if (!MW || wv == 0) {
    npairs = build_id_pairs<MM>(e, pairs);
    for (int q = lane; q < npairs; q += MFG_WAVE) {  // cells -> packed (x << 16 | y), agent independent
      const int cA = pairs.get(q, 0), cB = pairs.get(q, 1);
      pairs.set(q, 0, ((cA / W) << 16) | (cA % W));
      pairs.set(q, 1, ((cB / W) << 16) | (cB % W));
    }
    if (npairs > S->pairs_lds) mem_sync();
    if (MW && lane == 0) e.hdrp[MFG_HDR_N - 1] = npairs;  // an unused header slot of the LDS copy
  }
  if constexpr (MW) {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");  // the pair spill in HBM, then the LDS tables
    __syncthreads();
    npairs = uni(e.hdrp[MFG_HDR_N - 1]);
  }
  // first-visit table: (2d+1)^2 cells around the ray origin, min over visible (ray, point) of
  // ray << 5 | point (ray << 6 | point for rays longer than 32 points); it gives both the window visibility and the
  // dedupe order (Q14)
  uint32_t* fv = LR ? (uint32_t*)(S->obs_pool + (size_t)slot * (size_t)S->obs_slot_bytes)
                    : (uint32_t*)(e.scratch + 3 * S->pairs_lds + (MW ? wv * (S->lds_obs_wave >> 2) : 0));
  const int fw = 2 * fr + 1;
  uint8_t* wsup = (uint8_t*)(fv + S->fv_words);  // [dd] window cells whose wall or door the dedupe suppressed
  const int nsup4 = (dd + 3) >> 2;
  // dirt suppression bitmap for groups wider than a wave: after the per-lane sink words of the ray walk
  tu32* dsup = (tu32*)((uint32_t*)(wsup + ((dd + 15) & ~15)) + MFG_WAVE);
  const int ndsup = S->dirt_cap >> 5;
  // agents on each window cell: [dd][2] u32 (bit b = agent b), filled by a lane-per-agent scatter. Specs with more
  // than 64 agents (wide) always take the long-ray render (mfg_create), whose tables have a second [dd][2] table for
  // agents 64..127 (amw2); the other renders compile no wide code (their register budget is the C2-C5 one).
  tu32* amw = dsup + ndsup;
  const bool wide = LR && S->A > MFG_WAVE;
  tu32* amw2 = amw + 2 * dd;
  // window dirt map (specs with dirt): per window cell 1 + the index of the last present, non-suppressed pile on
  // it, built per agent from the pile table (lane = pile), so the placement reads a cell's pile instead of
  // scanning every pile per 64-cell block (C5: up to 384 piles)
  tu32* wdirt = amw + (wide ? 4 : 2) * dd;
  // packed mode: queue of the agent row's nonzero entries awaiting the fused projection ([64] flat index, [64] value);
  // the weight rows of up to 4 entries are loaded together, so their L2 latencies overlap instead of chaining
  tu32* pq = wdirt + (DIRT ? dd : 0);
  // FLAT: per window cell the stashed tag word (placement, then the flattened pass that stores the dense block or
  // queues the packed entries)
  // (packed: from windows wider than a wave on, pomdp_r >= 4 / rays of >= 10 points, where a layer's per-layer ballots
  // cover a partial second block: C4 fused projection 8.9 -> 10.5M env-steps/s; C3's 49-cell windows stay per layer,
  // 34.97 vs 34.3M flattened, profiles/r05_packed_flat_ab.json)
  // (dense and packed: only up to MFG_OBS_FLAT_MAXPTS ray points; C5's 18-point rays with 17 x 17 windows measured
  // k_obs 93 -> 110 ms flattened, profiles/r05_c5_flat_ab.json)
  constexpr bool FLAT = MFG_OBS_FLAT && (LR || MAXPTS <= MFG_OBS_FLAT_MAXPTS) &&
                        (PK == 0 || (MFG_OBS_FLAT_PK && (LR || MAXPTS > 8)));
  tu32* ctag = pq + 2 * MFG_WAVE;
  constexpr bool has_dirt = DIRT;  // S->dirt_cap != 0 (a template parameter: the register budget of k_obs)
  const float invW = 1.0f / (float)W;
  // lane-distributed copies of the small tables (uniform loops read them with v_readlane); agents 64.. of wide specs
  // are read from the record image per agent
  const int agp = lane < A ? e.agpos()[lane] : -1;
  const int org_l = lane < A ? (frozen ? e.forg()[lane] : agp) : -1;
  const int nT = e.H(H_N_DIRT);
  const int npass = (S->nrays + MFG_WAVE - 1) / MFG_WAVE;
  const int pA0 = lane < npairs ? pairs.get(lane, 0) : 0, pB0 = lane < npairs ? pairs.get(lane, 1) : 0;
  // agent and ray-origin coordinates: one vector division per render, read per agent with v_readlane
  const int agx = agp / W, agy = agp % W, orgx = org_l / W, orgy = org_l % W;
  // the first pass's rays are agent independent: loaded once per render, not once per agent, where the
  // registers they then hold across the agent loop do not cost occupancy (short rays, dense obs)
  constexpr bool HOIST_RAYS = !LR && MAXPTS <= 8 && PK == 0;  // (packed renders: per agent, measured faster)
  constexpr bool PREFETCH_RS = !LR && MAXPTS <= 8 && PK != 2;
  RayLane<RMP> ray0;
  if constexpr (HOIST_RAYS) ray0.load(S, lane);
  // ... and their static light-blocking words are fetched one agent ahead (an L2 round trip behind a
  // dependent cell_f load, hidden under the previous agent's dedupe and placement)
  int pf_ofl = -1;
  uint32_t pf_b = 0, pf_c = 0, pf_d = 0;
  auto rs_fetch = [&](int ag) {
    const int og = (!LR || ag < MFG_WAVE) ? rl(orgx, ag) * W + rl(orgy, ag) : uni(frozen ? e.forg()[ag] : e.agpos()[ag]);
    pf_ofl = S->ray_static ? uni((int)S->cell_f[og]) : -1;
    if (pf_ofl >= 0) {
      const bool has = lane < S->nrays;
      const uint32_t* rs = S->ray_static + ((size_t)pf_ofl * S->nrays + (has ? lane : 0)) * 3;
      pf_b = has ? rs[0] : 0u;
      pf_c = has ? rs[1] : 0u;
      pf_d = has ? rs[2] : 0u;
    }
  };
  if constexpr (PREFETCH_RS) rs_fetch(MW ? wv : 0);
  for (int a = MW ? wv : 0; a < A; a += MW ? nwv : 1) {
    int apos, ax, ay, ox, oy;
    if (!LR || a < MFG_WAVE) {
      apos = rl(agp, a);
      ax = rl(agx, a); ay = rl(agy, a);
      ox = rl(orgx, a); oy = rl(orgy, a);
    } else {  // agents 64..127 of a wide spec
      apos = uni(e.agpos()[a]);
      const int og = frozen ? uni(e.forg()[a]) : apos;
      ax = apos / W; ay = apos - ax * W;
      ox = og / W; oy = og - ox * W;
    }
    const int wx0 = full ? 0 : ax - S->r, wy0 = full ? 0 : ay - S->r;
    // origin floor index (static table)
    const int ofl = PREFETCH_RS ? pf_ofl : (S->ray_static ? uni((int)S->cell_f[ox * W + oy]) : -1);
    for (int i = lane; i < S->fv_words; i += MFG_WAVE) fv[i] = 0xFFFFFFFFu;
    for (int i = lane; i < nsup4; i += MFG_WAVE) ((uint32_t*)wsup)[i] = 0u;
    for (int i = lane; i < ndsup; i += MFG_WAVE) dsup[i] = 0u;
    for (int i = lane; i < (wide ? 4 : 2) * dd; i += MFG_WAVE) amw[i] = 0u;
    if (has_dirt)
      for (int i = lane; i < dd; i += MFG_WAVE) wdirt[i] = 0u;
    tbl_sync<LR>();
    if (lane < A) {  // scatter the agents into the window's agent masks
      const int wx = agx - wx0, wy = agy - wy0;
      if ((unsigned)wx < (unsigned)oh && (unsigned)wy < (unsigned)ow)
        atomicOr((uint32_t*)&amw[2 * (wx * ow + wy) + (lane >> 5)], 1u << (lane & 31));
    }
    if (wide && lane + MFG_WAVE < A) {  // agents 64..127
      const int p2 = e.agpos()[lane + MFG_WAVE];
      const int wx = p2 / W - wx0, wy = p2 % W - wy0;
      if ((unsigned)wx < (unsigned)oh && (unsigned)wy < (unsigned)ow)
        atomicOr((uint32_t*)&amw2[2 * (wx * ow + wy) + (lane >> 5)], 1u << (lane & 31));
    }
    // ---- ray walk (lane = ray, 64 rays per pass): blocking bits first, then the walk on bitmasks ----
    if constexpr (LR) {
      // long rays: each lane walks its ray in 32-point segments (points from the 16-bit table, dx | dy << 16),
      // carrying whether the walk has stopped and the previous point (the diagonal cut of a segment's first point);
      // per segment the same branch-free walk as below, first-visit rank = ray << 8 | point
      for (int pass = 0; pass < npass; pass++) {
        const int ray_id = pass * MFG_WAVE + lane;
        const bool has = ray_id < S->nrays;
        const int len = has ? (int)S->ray_len[ray_id] : 0;
        const uint32_t* rp = S->ray_pts16 + (size_t)(has ? ray_id : 0) * S->lrpts;
        uint32_t* sink = (uint32_t*)(wsup + ((dd + 15) & ~15)) + lane;
        bool stopped = false;
        int pdx = 0, pdy = 0;
        for (int s0 = 0; s0 < S->lrpts; s0 += 32) {
          uint32_t pt[32];
#pragma unroll
          for (int q = 0; q < 32; q++) pt[q] = rp[s0 + q];
          uint32_t blkm = 0u, cutm = 0u;
#pragma unroll
          for (int q = 0; q < 32; q++) {
            const int dx = (int)(int16_t)(pt[q] & 0xFFFFu), dy = (int)(int16_t)(pt[q] >> 16);
            const int qdx = q ? (int)(int16_t)(pt[q - 1] & 0xFFFFu) : pdx, qdy = q ? (int)(int16_t)(pt[q - 1] >> 16) : pdy;
            const int x = ox + dx, y = oy + dy;
            blkm |= light_block_bf<MM>(e, x, y) ? (1u << q) : 0u;
            // a diagonal step from the previous point is cut when both orthogonal neighbours block light
            // (ray_caster.py:89-96)
            const bool dg = (s0 + q > 0) & (dx != qdx) & (dy != qdy);
            const bool c = dg & light_block_bf<MM>(e, x, oy + qdy) & light_block_bf<MM>(e, ox + qdx, y);
            cutm |= c ? (1u << q) : 0u;
          }
          pdx = (int)(int16_t)(pt[31] & 0xFFFFu);
          pdy = (int)(int16_t)(pt[31] >> 16);
          const int rem = len - s0;
          const uint32_t lenm = rem >= 32 ? 0xFFFFFFFFu : (rem <= 0 ? 0u : ((1u << rem) - 1u));
          const uint32_t stopm = (blkm | cutm) & lenm;
          const uint32_t walked = stopped ? 0u : (stopm ? (((stopm & (0u - stopm)) << 1) - 1u) & lenm : lenm);
          const uint32_t vism = walked & ~cutm;
          stopped |= stopm != 0u;
#pragma unroll
          for (int q = 0; q < 32; q++) {
            const int dx = (int)(int16_t)(pt[q] & 0xFFFFu), dy = (int)(int16_t)(pt[q] >> 16);
            const bool vq = ((vism >> q) & 1u) && (s0 + q > 0);  // the origin (point 0) is stored once below
            atomicMin(vq ? &fv[(dx + fr) * fw + dy + fr] : sink, (uint32_t)((ray_id << 8) + s0 + q));
          }
        }
      }
    } else
    for (int pass = 0; pass < npass; pass++) {
      const int ray_id = pass * MFG_WAVE + lane;
      RayLane<RMP> ray;
      if (HOIST_RAYS && pass == 0) ray = ray0;
      else ray.load(S, ray_id);
      // branch-free: every point tests its cell and (from p = 1) both corner cells; the static diagonal
      // mask keeps the corner test only on diagonal steps: cut when both orthogonal neighbours block
      // light (ray_caster.py:89-96)
      typedef typename RayLane<RMP>::PM PM;
      constexpr int NB = 8 * (int)sizeof(PM);
      PM blkm = 0, cutm = 0;
      if (RMP <= 32 && ofl >= 0) {  // (no static table for rays longer than 32 points: ofl is -1 there)
        // the wall part from the per-origin table; only points next to doors are tested here (the door's
        // present/closed state lives in the cell map)
        uint32_t dyn;
        if (PREFETCH_RS && pass == 0) {
          blkm = pf_b;
          cutm = pf_c;
          dyn = pf_d;
          if (a + (MW ? nwv : 1) < A) rs_fetch(a + (MW ? nwv : 1));
        } else {
          const bool has = ray_id < S->nrays;
          const uint32_t* rs = S->ray_static + ((size_t)ofl * S->nrays + (has ? ray_id : 0)) * 3;
          blkm = has ? rs[0] : 0u;
          cutm = has ? rs[1] : 0u;
          dyn = has ? rs[2] : 0u;
        }
        while (dyn) {
          const int p = __ffs((int)dyn) - 1;
          dyn &= dyn - 1;
          const int8_t* pt = S->ray_pts + ((size_t)ray_id * S->maxpts + p) * 2;
          const int x = ox + pt[0], y = oy + pt[1];
          blkm |= light_block_bf<MM>(e, x, y) ? ((PM)1 << p) : (PM)0;
          if (p > 0 && ((ray.diag >> p) & 1u)) {
            const bool c = light_block_bf<MM>(e, x, oy + pt[-1]) & light_block_bf<MM>(e, ox + pt[-2], y);
            cutm |= c ? ((PM)1 << p) : (PM)0;
          }
        }
      } else {
#pragma unroll
        for (int p = 0; p < RMP; p++) {
          const int x = ox + ray.dx(p), y = oy + ray.dy(p);
          blkm |= light_block_bf<MM>(e, x, y) ? ((PM)1 << p) : (PM)0;
          if (p > 0) {
            const bool c = light_block_bf<MM>(e, x, oy + ray.dy(p - 1)) & light_block_bf<MM>(e, ox + ray.dx(p - 1), y);
            cutm |= c ? ((PM)1 << p) : (PM)0;
          }
        }
      }
      cutm &= ray.diag;
      // points walked: up to and including the first blocking/cut point, within the ray length
      const PM lenm = ray.len >= NB ? ~(PM)0 : (((PM)1 << ray.len) - (PM)1);
      const PM stopm = (blkm | cutm) & lenm;
      const PM walked = stopm ? (((stopm & ((PM)0 - stopm)) << 1) - (PM)1) & lenm : lenm;
      // points outside the grid are recorded too: nothing is there (no entity, no wall), so their
      // first-visit entries are never read (placement tests the grid bounds, pairs are in-grid cells)
      const PM vism = walked & ~cutm;
      uint32_t* sink = (uint32_t*)(wsup + ((dd + 15) & ~15)) + lane;
      // point 0 of every ray is the origin (checked at mfg_create) and always visible: its entry is
      // ray 0's rank 0, stored once below instead of a 64-lane same-address atomic
#pragma unroll
      for (int p = 1; p < RMP; p++)
        atomicMin(((vism >> p) & 1u) ? &fv[(ray.dx(p) + fr) * fw + ray.dy(p) + fr] : sink,
                  (uint32_t)((ray_id << RayLane<RMP>::RSH) + p));
    }
    if (lane == 0) fv[fr * fw + fr] = 0u;
    tbl_sync<LR>();
    // ---- identifier dedupe: of two visible entities with equal identifiers the later first visit loses
    SupT<tu32> sup;
    sup.items = sup.pods = sup.drops = sup.dests = sup.machines = sup.maints = 0;
    sup.wx0 = wx0; sup.wy0 = wy0; sup.oh = oh; sup.ow = ow; sup.W = W;
    sup.wsup = wsup;
    sup.dsup = dsup;
    for (int q0 = 0; q0 < npairs; q0 += MFG_WAVE) {
      const int q = q0 + lane;
      // the first pass's pair cells stay in registers across agents (the usual single pass)
      const int pA = q0 == 0 ? pA0 : (q < npairs ? pairs.get(q, 0) : 0);
      const int pB = q0 == 0 ? pB0 : (q < npairs ? pairs.get(q, 1) : 0);
      const int xA = (pA >> 16) - ox + fr, yA = (pA & 0xFFFF) - oy + fr;
      const int xB = (pB >> 16) - ox + fr, yB = (pB & 0xFFFF) - oy + fr;
      const bool nearq = (q < npairs) & ((unsigned)xA < (unsigned)fw) & ((unsigned)yA < (unsigned)fw) &
                         ((unsigned)xB < (unsigned)fw) & ((unsigned)yB < (unsigned)fw);
      const uint32_t rA0 = fv[nearq ? xA * fw + yA : 0], rB0 = fv[nearq ? xB * fw + yB : 0];
      const uint32_t rA = nearq ? rA0 : 0xFFFFFFFFu, rB = nearq ? rB0 : 0xFFFFFFFFu;
      u64 hm = ballot(rA != 0xFFFFFFFFu && rB != 0xFFFFFFFFu);
      while (hm) {
        const int L = ffs64(hm);
        hm &= hm - 1;
        const int qq = q0 + L;
        const int codes = pairs.get(qq, 2);  // codeA | codeB << 16
        if (rl((int)rA, L) < rl((int)rB, L)) sup_add(sup, (codes >> 16) & 0xFFFF, rl(pB, L), lane);
        else sup_add(sup, codes & 0xFFFF, rl(pA, L), lane);
      }
    }
    tbl_sync<LR>();
    if (has_dirt) {
      // clean_up piles on window cells, in table order: the last one wins (the sequential scan it replaces
      // kept the last matching pile's amount); cell / W through a float reciprocal (exact for cells < 2^16)
      for (int b = 0; b < nT; b += MFG_WAVE) {
        const int i = b + lane;
        const int w = i < nT ? e.dirtpos()[i] : 0;
        const int c = EW_POS(w);
        const int cx = (int)(((float)c + 0.5f) * invW), cy = c - cx * W;
        const int px = cx - wx0, py = cy - wy0;
        if (i < nT && (w & EW_PRESENT) && c != EW_NOPOS && (unsigned)px < (unsigned)oh && (unsigned)py < (unsigned)ow &&
            !sup.dirt_sup(i))
          atomicMax((uint32_t*)&wdirt[px * ow + py], (uint32_t)(i + 1));
      }
      tbl_sync<LR>();
    }
    OT* out_a = PK ? nullptr : out_env + (size_t)a * S->obs_agent_stride;
    const int nl = S->s.n_layers[a];
    // the agent's layer records, lane l = layer l (read per layer with v_readlane: no scalar load waited on
    // inside the placement loop); unit tags < 16 bits, flags above them
    uint32_t lr_tf = 0, lr_alo = 0, lr_ahi = 0;
    {
      const MfgLayerRec CS* lr = (const MfgLayerRec CS*)S->lrec + (size_t)a * S->lmax;
      if (lane < nl) {
        lr_tf = (lr[lane].unit_tags & 0xFFFFu) | (lr[lane].flags << 16);
        lr_alo = (uint32_t)lr[lane].agent_bits;
        lr_ahi = (uint32_t)(lr[lane].agent_bits >> 32);
      }
    }
    // packed mode: entry count so far and the projection accumulators (lane j holds outputs j, 64 + j, ...)
    int qbase = 0, nq = 0;  // entries flushed so far; entries in the queue
    float acc[MFG_MAX_EMB / MFG_WAVE];
    // flush the queued entries (in flat index order with FLAT, else (block, layer, cell) order): the stored row slots qbase + t < cap (one
    // coalesced store per array instead of one partial store per layer block), then the projection
    // acc[j] += val_t * wt[idx_t][j]
    auto flush = [&]() {
      const int qi = (int)pq[lane], qv = (int)pq[MFG_WAVE + lane];  // lane t holds entry t
      if (pk.idx && lane < nq && qbase + lane < pk.cap) {
        pk.idx[(size_t)a * pk.cap + qbase + lane] = (uint16_t)qi;
        pk.val[(size_t)a * pk.cap + qbase + lane] = __int_as_float(qv);
      }
      for (int t = 0; PK == 2 && pk.emb && t < nq; t += 4) {
        float w4[4][MFG_MAX_EMB / MFG_WAVE], v4[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
          const int tt = min(t + u, nq - 1);
          v4[u] = t + u < nq ? __int_as_float(rl(qv, tt)) : 0.0f;
          const float* wr = pk.wt + (size_t)rl(qi, tt) * pk.E;
#pragma unroll
          for (int q = 0; q < MFG_MAX_EMB / MFG_WAVE; q++) {
            const int j = q * MFG_WAVE + lane;
            w4[u][q] = (q * MFG_WAVE < pk.E && j < pk.E) ? wr[j] : 0.0f;
          }
        }
#pragma unroll
        for (int u = 0; u < 4; u++)
          if (t + u < nq)
#pragma unroll
            for (int q = 0; q < MFG_MAX_EMB / MFG_WAVE; q++) acc[q] = __builtin_fmaf(v4[u], w4[u][q], acc[q]);
      }
      qbase += nq;
      nq = 0;
    };
    if constexpr (PK == 2) {
#pragma unroll
      for (int q = 0; q < MFG_MAX_EMB / MFG_WAVE; q++) {
        const int j = q * MFG_WAVE + lane;
        acc[q] = (pk.bias && j < pk.E) ? pk.bias[j] : 0.0f;
      }
    }
    // ---- placement (lane = window cell, 64 cells per pass): tag bits from the cell map ----
    for (int w0 = 0; w0 < dd; w0 += MFG_WAVE) {
      // dense (and FLAT): lanes past the window repeat the last window cell (its value, to its address), so the layer
      // stores need no exec mask; the per-layer packed placement keeps them out (its ballots count entries)
      const int wi = PK && !FLAT ? w0 + lane : min(w0 + lane, dd - 1);
      const bool inwin = PK && !FLAT ? wi < dd : true;
      // wi / d and wi % d through a float reciprocal (exact: (wi + 0.5) / d is >= 0.5 / d away from an integer
      // and the product's error is <= (wi + 0.5) / d * 2^-23, below that for wi < 2^22); the tests below are branch-free, every LDS
      // read has a valid clamped address and its result is masked
      const int wq = (int)(((float)wi + 0.5f) * invw), wr = wi - wq * ow;
      const int x = wx0 + wq, y = wy0 + wr;
      const int lx = x - ox + fr, ly = y - oy + fr;
      const bool inb = inwin & ((unsigned)x < (unsigned)H) & ((unsigned)y < (unsigned)W) &
                       ((unsigned)lx < (unsigned)fw) & ((unsigned)ly < (unsigned)fw);
      const bool v = inb & (fv[inb ? lx * fw + ly : 0] != 0xFFFFFFFFu);
      const int cell = v ? x * W + y : 0;
      // the cell-map read does not wait for the visibility read: its address is clamped on the bounds alone
      const uint32_t mraw = cmap_at<MM>(e, inb ? x * W + y : 0);
      const uint32_t m = v ? mraw : 0u;
      // CM_WALL | CM_DOOR when the cell's wall or door lost an identifier dedupe (a cell holds at most one of the two)
      const uint32_t wall_sup = wsup[inwin ? wi : 0];
      // bit t = tag t (< 16) has a (not suppressed) entity here: the cell-map bits are the tag bits
      uint32_t tags = (m & ~wall_sup) & (CM_WALL | CM_DOOR | CM_ITEM | CM_POD | CM_DROP | CM_DIRT | CM_DEST);
      if (MM) tags |= (m >> 1) & ((1u << MFG_TAG_MACHINES) | (1u << MFG_TAG_MAINTAINERS));
      // identifier-dedupe suppressions (rare): recompute the affected tags from the entity tables
      auto resup = [&](const int* tbl, int n, u64 sm, int tag, bool dest) {
        if (!sm) return;
        bool any = false;
        for (int i = 0; i < n; i++) {
          const int w = uni(tbl[i]);
          any |= v && EW_POS(w) == cell && (w & EW_PRESENT) && !((sm >> i) & 1) && !(dest && (w & EW_REACHED));
        }
        tags = any ? (tags | (1u << tag)) : (tags & ~(1u << tag));
      };
      resup(e.items(), e.H(H_N_ITEMS), sup.items, MFG_TAG_ITEMS, false);
      resup(e.pods(), e.H(H_N_PODS), sup.pods, MFG_TAG_PODS, false);
      resup(e.drops(), e.H(H_N_DROPS), sup.drops, MFG_TAG_DROPOFFS, false);
      resup(e.dests(), e.H(H_N_DESTS), sup.dests, MFG_TAG_DESTS, true);
      if (MM && S->mmax) resup(e.machines(), e.H(H_N_MACHINES), sup.machines, MFG_TAG_MACHINES, false);
      if (MM && S->kmax) resup(e.maints(), e.H(H_N_MAINTS), sup.maints, MFG_TAG_MAINTAINERS, false);
      double dirt_amt = 0.0;
      if (has_dirt) {  // amount of the last non-suppressed pile on the cell (window dirt map)
        const uint32_t di = v ? wdirt[inwin ? wi : 0] : 0u;
        dirt_amt = di ? e.dirtamt()[di - 1] : 0.0;
        tags = di ? (tags | (1u << MFG_TAG_DIRT)) : (tags & ~(1u << MFG_TAG_DIRT));
      }
      const int wic = inwin ? wi : 0;
      const u64 amraw = (u64)amw[2 * wic] | ((u64)amw[2 * wic + 1] << 32);
      const u64 amask = v ? amraw : 0ull;
      // tag value: entity encodings (walls/agents/items/pods/drop-offs/destinations 1, doors 0.6666 closed /
      // 0.4444 open, dirt = amount)
      auto tagv = [&](int tag) -> double {
        if (wide && tag >= MFG_TAG_AGENT0 + MFG_WAVE) {  // agents 64..127: the second mask table
          const int b = tag - MFG_TAG_AGENT0 - MFG_WAVE;
          return (v && ((amw2[2 * wic + (b >> 5)] >> (b & 31)) & 1u)) ? 1.0 : 0.0;
        }
        if (tag >= MFG_TAG_AGENT0) return ((amask >> (tag - MFG_TAG_AGENT0)) & 1) ? 1.0 : 0.0;
        if (!((tags >> tag) & 1u)) return 0.0;
        if (tag == MFG_TAG_DOORS) return (m & CM_DCLOSED) ? 0.6666 : 0.4444;
        if (tag == MFG_TAG_DIRT) return dirt_amt;
        if (tag == MFG_TAG_MACHINES) return (double)S->s.machine_pause;  // idle forever: encoding 15 (Q18)
        return 1.0;
      };
      if constexpr (FLAT) {  // stash: the flattened pass below writes the layers (each lane only its own cell here)
        ctag[wi] = tags | ((m & CM_DCLOSED) ? CT_CLOSED : 0u);
        amw[2 * wi] = (uint32_t)amask;
        amw[2 * wi + 1] = (uint32_t)(amask >> 32);
        if (wide) {
          const uint32_t w0v = amw2[2 * wi], w1v = amw2[2 * wi + 1];
          amw2[2 * wi] = v ? w0v : 0u;
          amw2[2 * wi + 1] = v ? w1v : 0u;
        }
        if (has_dirt) wdirt[wi] = v ? wdirt[wi] : 0u;
        continue;
      }
      OT* op = PK ? nullptr : out_a + wi;  // this lane's cell of layer l: op + l * dd (advanced per layer)
      for (int l = 0; l < nl; l++, op += PK ? 0 : dd) {
        const uint32_t tf = (uint32_t)rl((int)lr_tf, l);
        const uint32_t ut = tf & 0xFFFFu, fl = tf >> 16;
        const uint64_t ab = (uint64_t)(uint32_t)rl((int)lr_alo, l) | ((uint64_t)(uint32_t)rl((int)lr_ahi, l) << 32);
        int cnt = popc(tags & ut) + popc(amask & ab);
        if (wide) {  // agents 64..127: the layer's second agent word (uniform load) against the second mask table
          const uint64_t ab2 = S->lrec_ab2[(size_t)a * S->lmax + l];
          const u64 am2 = v ? ((u64)amw2[2 * wic] | ((u64)amw2[2 * wic + 1] << 32)) : 0ull;
          cnt += popc(am2 & ab2);
        }
        OT out = (OT)cnt;  // a small count: exact in OT
        if (fl) {
          double val = 0.0;
          if (fl & LR_DOOR) {
            val = tagv(MFG_TAG_DOORS);
          } else if (fl & LR_DIRT) {
            val = tagv(MFG_TAG_DIRT);
          } else if (fl & LR_MACHINE) {
            val = tagv(MFG_TAG_MACHINES);
          } else if (fl & LR_ORDERED) {
            const int nc = S->s.combined_n[a];
            for (int q = 0; q < nc; q++) {
              const double tv = tagv(S->s.combined_tags[a][q]);
              val = q == 0 ? tv : val + tv;
            }
          } else if (fl & LR_BATTERY) {
            val = wi == 0 ? (frozen ? e.fbat()[a] : e.bat()[a]) : 0.0;
          } else {  // LR_GLOBALPOS
            const int gp = frozen ? e.fgp()[a] : apos;
            val = wi == 0 ? (double)(gp / W) / (double)H : (wi == 1 ? (double)(gp % W) / (double)W : 0.0);
          }
          out = (OT)val;
        }
        if constexpr (PK) {
          // nonzero entries of this layer's 64-cell block, in lane order; the projection walks them in
          // the same order (uniform loop, lane = output feature, coalesced rows of wt)
          const float fv = (float)out;
          const bool nz = inwin && fv != 0.0f;
          const u64 nzm = ballot(nz);
          const int base = l * dd + w0;
          if (nzm) {
            const int nb = popc(nzm);
            if (nq + nb > MFG_WAVE) {
              tbl_sync<LR>();
              flush();
            }
            if (nz) {
              const int qpos = nq + mbcnt(nzm);
              pq[qpos] = (uint32_t)(base + lane);
              pq[MFG_WAVE + qpos] = (uint32_t)__float_as_int(fv);
            }
            nq += nb;
          }
          continue;
        }
        // non-temporal: the obs stream is not re-read by this GPU (k_obs 0.500 -> 0.493 ms, k_logic
        // 0.298 -> 0.291 ms at C3: less L2 pollution). WRITE_SIZE counts 1.34x the algorithmic obs bytes
        // for these stores (1.00x with MFG_OBS_NT=0): the 49-lane layer rows are not 64-B aligned.
        // Packing rows into aligned 64-lane stores (ds_bpermute) cut that to 1.14x but cost 67 VGPRs
        // and k_obs 0.494 -> 0.543 ms, so it was dropped (k_obs).
#ifndef MFG_OBS_PLAIN_PTS
#define MFG_OBS_PLAIN_PTS 12
#endif
        // multi-wave render with short rays (<= MFG_OBS_PLAIN_PTS points: windows up to 11 x 11, C4's 9 x 9 rows of
        // 648 B in f64): plain stores, which merge a row's partial lines with the next layer's in L2 before they go
        // to HBM (C4 k_obs f64 2.63 -> 1.78 ms, f32 1.87 -> 1.39). Longer rows (C5's 17 x 17: 79.8 -> 87.6 ms plain)
        // and the single-wave render (C3: the next k_logic's records stay in L2, 0.132 vs 0.146 ms) keep
        // non-temporal stores. Compile-time: a run-time choice between the two stores gets merged into one store
        // without the non-temporal hint.
        if constexpr (MW && MAXPTS <= MFG_OBS_PLAIN_PTS) {
          if (inwin) *op = out;
        } else {
          if (inwin) __builtin_nontemporal_store(out, op);
        }
      }
    }
    if constexpr (FLAT) {
      // the agent's [nl][dd] block as consecutive runs of 64 values: lane = element el = l * dd + c (l, c by a float
      // reciprocal, exact for el < 2^22), the cell's stashed words from LDS, the layer record of layer l from lane l
      // (ds_bpermute); the value formulas are the per-layer placement's. Lanes past the block repeat its last value.
      // Packed: one ballot per 64 elements queues the nonzero ones, so a row's entries come in flat index order.
      tbl_sync<LR>();
      const int ne = nl * dd;
      const float invdd = 1.0f / (float)dd;
      for (int e0 = 0; e0 < ne; e0 += MFG_WAVE) {
        const int el = min(e0 + lane, ne - 1);
        const int l = (int)(((float)el + 0.5f) * invdd), c = el - l * dd;
        const uint32_t ct = ctag[c];
        const u64 am = (u64)amw[2 * c] | ((u64)amw[2 * c + 1] << 32);
        const uint32_t tf = bperm(l, lr_tf);
        const uint64_t ab = (uint64_t)bperm(l, lr_alo) | ((uint64_t)bperm(l, lr_ahi) << 32);
        const uint32_t ut = tf & 0xFFFFu, fl = tf >> 16;
        int cnt = popc(ct & ut) + popc(am & ab);
        if (wide) {  // agents 64..127: layer l's second agent word (per-lane load) against the second mask table
          const uint64_t ab2 = S->lrec_ab2[(size_t)a * S->lmax + l];
          cnt += popc(((u64)amw2[2 * c] | ((u64)amw2[2 * c + 1] << 32)) & ab2);
        }
        OT out = (OT)cnt;  // a small count: exact in OT
        if (fl) {
          auto tagv = [&](int tag) -> double {
            if (wide && tag >= MFG_TAG_AGENT0 + MFG_WAVE) {  // agents 64..127: the second mask table
              const int b = tag - MFG_TAG_AGENT0 - MFG_WAVE;
              return ((amw2[2 * c + (b >> 5)] >> (b & 31)) & 1u) ? 1.0 : 0.0;
            }
            if (tag >= MFG_TAG_AGENT0) return ((am >> (tag - MFG_TAG_AGENT0)) & 1) ? 1.0 : 0.0;
            if (!((ct >> tag) & 1u)) return 0.0;
            if (tag == MFG_TAG_DOORS) return (ct & CT_CLOSED) ? 0.6666 : 0.4444;
            if (tag == MFG_TAG_DIRT) {
              const uint32_t di = has_dirt ? (uint32_t)wdirt[c] : 0u;
              return di ? e.dirtamt()[di - 1] : 0.0;
            }
            if (tag == MFG_TAG_MACHINES) return (double)S->s.machine_pause;  // idle forever: encoding 15 (Q18)
            return 1.0;
          };
          double val = 0.0;
          if (fl & LR_DOOR) {
            val = tagv(MFG_TAG_DOORS);
          } else if (fl & LR_DIRT) {
            val = tagv(MFG_TAG_DIRT);
          } else if (fl & LR_MACHINE) {
            val = tagv(MFG_TAG_MACHINES);
          } else if (fl & LR_ORDERED) {
            const int nc = S->s.combined_n[a];
            for (int q = 0; q < nc; q++) {
              const double tv = tagv(S->s.combined_tags[a][q]);
              val = q == 0 ? tv : val + tv;
            }
          } else if (fl & LR_BATTERY) {
            val = c == 0 ? (frozen ? e.fbat()[a] : e.bat()[a]) : 0.0;
          } else {  // LR_GLOBALPOS
            const int gp = frozen ? e.fgp()[a] : apos;
            val = c == 0 ? (double)(gp / W) / (double)H : (c == 1 ? (double)(gp % W) / (double)W : 0.0);
          }
          out = (OT)val;
        }
        if constexpr (PK) {
          const float fv = (float)out;
          const bool nz = e0 + lane < ne && fv != 0.0f;
          const u64 nzm = ballot(nz);
          if (nzm) {
            const int nb = popc(nzm);
            if (nq + nb > MFG_WAVE) {
              tbl_sync<LR>();
              flush();
            }
            if (nz) {
              const int qpos = nq + mbcnt(nzm);
              pq[qpos] = (uint32_t)el;
              pq[MFG_WAVE + qpos] = (uint32_t)__float_as_int(fv);
            }
            nq += nb;
          }
          continue;
        }
        // non-temporal for every render: the 64-value runs leave at most the two edge lines of a run partial, so
        // the L2 merge that made plain stores pay for the per-layer rows of the multi-wave render is not needed
        // (C4 isolated k_obs 1.54 -> 1.36 ms, C4 10.72M -> 11.16M env-steps/s, profiles/r05_c4_flat_nt_ab.json)
        __builtin_nontemporal_store(out, out_a + el);
      }
    }
    if constexpr (PK) {
      if (nq) {
        tbl_sync<LR>();
        flush();
      }
      const int pcount = qbase;
      if (pk.idx)  // unused slots: idx 0 / val 0 (a fixed-width gather over the row stays exact)
        for (int i = pcount + lane; i < pk.cap; i += MFG_WAVE) {
          pk.idx[(size_t)a * pk.cap + i] = 0;
          pk.val[(size_t)a * pk.cap + i] = 0.0f;
        }
      if (pk.cnt && lane == 0) pk.cnt[a] = pcount;
      if (PK == 2 && pk.emb) {
#pragma unroll
        for (int q = 0; q < MFG_MAX_EMB / MFG_WAVE; q++) {
          const int j = q * MFG_WAVE + lane;
          if (q * MFG_WAVE < pk.E && j < pk.E) pk.emb[(size_t)a * pk.E + j] = acc[q];
        }
      }
    }
  }
}

// ------------------------------------------------------------------------------------------------
// one env-step (Factory.step, factory.py:189-220; Gamestate.tick, states.py:170-203)
// ------------------------------------------------------------------------------------------------
#define MFG_EV_MISC MFG_EV_MISC_N

template <bool RNG, bool MAINT, int NW>
__device__ void env_step(const Env& e, const int (&my_act)[NW], StepOut<NW>& o, int* scratch) {
  SpecP S = e.S;
  const int A = S->A;
#pragma unroll
  for (int h = 0; h < NW; h++) {
    o.my_rew[h] = 0.0; o.my_act_ev[h] = 0; o.my_watch_ev[h] = 0; o.my_slot[h] = -1; o.door_coll[h] = 0;
  }
  o.g_rew = 0.0; o.maint_coll = 0;
  o.respawn_items_value = -1; o.dirt_spawn_value = -1; o.dirt_spawn_valid = 0; o.door_autoclose = 0;
  o.done_mask = 0; o.dest_reached = 0; o.crashed = 0; o.done = 0;
  e.setH(H_STEP, e.H(H_STEP) + 1);
  e.setH(H_TOTAL_STEPS, e.H(H_TOTAL_STEPS) + 1);
  o.crashed = e.H(H_CRASHED);  // a crash the reset hit (or a crashed env stepped without a reset): done, no step
  wave_sync();
  const int a0 = o.crashed ? A : act_parallel<NW>(e, my_act, o);
  for (int a = a0; a < A && !o.crashed; a++) {
    if (uni(e.agpar()[a])) continue;  // paralyzed agents skip their action
    const int slot = agent_get(my_act, a);
    if (slot < 0 || slot >= S->s.n_actions[a]) { o.crashed = MFG_CRASH_ACTION; break; }  // IndexError upstream
    do_action<NW>(e, o, a, slot);
    agent_set(o.my_slot, a, e.lane, slot);
  }
  if (!o.crashed)
    for (int q = 0; q < S->n_ph[0] && !o.crashed; q++) rule_tick_step<RNG, MAINT, NW>(e, o, S->ph_rule[0][q], scratch);
  if (!o.crashed)
    for (int q = 0; q < S->n_ph[1] && !o.crashed; q++) rule_post_step<NW>(e, o, S->ph_rule[1][q]);
  if (!o.crashed)
    for (int q = 0; q < S->n_ph[2]; q++) rule_check_done<NW>(e, o, S->ph_rule[2][q]);
  // the step's membership-only shuffles stay as debt: paid by k_replay after the launch, or inline by
  // the next order-dependent consumer (spawn / reset)
  if (o.crashed || e.H(H_OVERFLOW)) {  // H_CRASHED keeps the reason (MFG_CRASH_*, include/mfg.h)
    o.crashed = o.crashed ? o.crashed : MFG_CRASH_CAPACITY;
    e.setH(H_CRASHED, o.crashed);
    o.done = 1;
  }
  wave_sync();
}

template <int NW>
__device__ __forceinline__ void write_step_outputs(const Env& e, const StepOut<NW>& o, size_t row, double* reward,
                                                   uint8_t* done, uint8_t* ev_act, uint8_t* ev_watch,
                                                   int32_t* ev_misc) {
  const int A = e.S->A;
#pragma unroll
  for (int h = 0; h < NW; h++) {
    const int a = h * MFG_WAVE + e.lane;
    if (a < A) {
      if (reward) reward[row * A + a] = o.my_rew[h] + o.g_rew;
      if (ev_act) ev_act[row * A + a] = (uint8_t)o.my_act_ev[h];
      if (ev_watch) ev_watch[row * A + a] = (uint8_t)o.my_watch_ev[h];
    }
  }
  if (e.lane == 0 && done) done[row] = (uint8_t)o.done;
  if (ev_misc) {  // one 16-lane store (lane k writes slot k) instead of 16 single-lane stores
    const int l = e.lane;
    int v = (int)(uint32_t)o.door_coll[0];
    v = l == 1 ? (int)(uint32_t)(o.door_coll[0] >> 32) : v;
    v = l == 2 ? o.respawn_items_value : v;
    v = l == 3 ? o.dirt_spawn_value : v;
    v = l == 4 ? o.dirt_spawn_valid : v;
    v = l == 5 ? o.dest_reached : v;
    v = l == 6 ? ((o.door_autoclose ? 1 : 0) | (o.crashed ? 2 : 0) | ((o.crashed & 0xFF) << 8)) : v;
    v = l == 7 ? o.done_mask : v;
    v = l == 8 ? e.hdr()[H_STEP] : v;
    v = l == 9 ? e.hdr()[H_EPISODE] : v;
    v = l == 10 ? (int32_t)(uint32_t)o.maint_coll : v;
    v = l == 11 ? (e.S->kmax ? e.hdr()[H_MAINT_BASE] : 0) : v;
    v = l == 12 ? (NW > 1 ? (int)(uint32_t)o.door_coll[NW - 1] : 0) : v;
    v = l == 13 ? (NW > 1 ? (int)(uint32_t)(o.door_coll[NW - 1] >> 32) : 0) : v;
    v = l == 14 ? (int32_t)(uint32_t)(o.maint_coll >> 32) : v;
    v = l == 15 ? 0 : v;
    static_assert(MFG_EV_MISC == 16, "ev_misc row width");
    if (e.lane < MFG_EV_MISC) ev_misc[row * MFG_EV_MISC + e.lane] = v;
  }
}

// ------------------------------------------------------------------------------------------------
// kernels: one wave per env, MFG_WPB waves per workgroup, (a prefix of) the env record image in
// dynamic LDS. One env-step is three launches over all envs, each sized for its own working set:
//   k_logic     actions + rules + rewards/done/events; LDS = record without MT/perm (the "lean" record)
//               unless the spec consumes the floor order inside a step (dirt spawns)
//   k_resetdone auto-reset of the envs that just finished (full record, early exit for the rest)
//   k_obs       observation render; LDS = lean record + cell map + id-collision pairs; read-only on state
// and k_replay pays the accumulated floor-shuffle debt once per mfg_step call.
// ------------------------------------------------------------------------------------------------
#define MFG_PAIRS_LDS 128    // identifier-collision pairs kept in the k_obs LDS slice
#define MFG_LDS_MAX 163840  // LDS bytes per CU on gfx950 (one workgroup may use all of it)
#define MFG_WPB 4  // waves (envs) per workgroup at most; fewer when a slice is large (wpb_for)
// k_logic<false, false> is SGPR-bound to 7 waves per SIMD (106 SGPRs); asking for 8 fits it in 78 SGPRs with one
// SGPR spill (C3: 0.1505 -> 0.1303 ms per launch). The same request on the dense k_obs spills ~90 SGPRs into VGPR
// lanes and made it slower (0.433 -> 0.451 ms), so k_obs keeps 7.
#define MFG_WPE_LOGIC(n) __attribute__((amdgpu_waves_per_eu(n)))
// the single-wave render (short rays) asks for 7 waves per SIMD. 8 (round 4 A/B): C3 f64 k_obs 0.4995 -> 0.495 ms,
// but C3 f32 0.399 -> 0.466 and C2 f64 0.032 -> 0.038 ms (84 SGPRs spilled into VGPR lanes, 2 VGPRs to scratch)

// full-record slice: [record][scratch][shuffle tables][BFS scratch if it fits]
__device__ __forceinline__ void env_full(SpecP S, uint8_t* slice, Env& e, long long env) {
  e.S = S;
  e.lds = slice;
  e.scratch = (int*)(slice + S->L.size);
  e.stab = (uint32_t*)(slice + S->L.size + S->scratch_bytes);
  e.cmap = nullptr;
  e.bfs = S->bfs_pool ? S->bfs_pool + (size_t)env * S->bfs_bytes : (S->bfs_off ? slice + S->bfs_off : nullptr);
  e.hdrp = (int*)(slice + S->L.o_hdr);
  e.lane = lane_id();
  for (int i = e.lane; i < MFG_STAB_N; i += MFG_WAVE) e.stab[i] = 0u;
}
__device__ __forceinline__ void rec_copy(uint8_t* dst, const uint8_t* src, int bytes, int lane) {
  const int n16 = bytes >> 4;
  for (int i = lane; i < n16; i += MFG_WAVE) ((uint4*)dst)[i] = ((const uint4*)src)[i];
}
// The step prefix [0, o_logic) without the dirt slots at or past nd (the live pile count): [0, pos + 4 nd),
// [id, id + 4 nd), [battery, amount + 8 nd), [pcg, o_logic), each widened to 16 B. The widening and the overlaps only
// touch dead slots, which a lean step neither reads nor writes, so they go back unchanged.
#ifndef MFG_LOGIC_TRIM
#define MFG_LOGIC_TRIM 1
#endif
// dirt = false (the write-back of a step that changed no dirt table, H_DIRT_TOUCH): the dirt slots are skipped; a
// 16-B chunk shared with a neighbouring field goes back with its staged (unchanged) dirt bytes
__device__ __forceinline__ void prefix_copy(uint8_t* dst, const uint8_t* src, SpecP S, int nd, int lane,
                                            bool dirt = true) {
  auto seg = [&](int b, int end) {
    b &= ~15;
    end = (end + 15) & ~15;
    for (int i = b + 16 * lane; i < end; i += 16 * MFG_WAVE) *(uint4*)(dst + i) = *(const uint4*)(src + i);
  };
  if (dirt) {
    seg(0, S->L.o_dirt_pos + 4 * nd);
    seg(S->L.o_dirt_id, S->L.o_dirt_id + 4 * nd);
    seg(S->L.o_battery, S->L.o_dirt_amt + 8 * nd);
  } else {
    seg(0, S->L.o_dirt_pos);
    seg(S->L.o_battery, S->L.o_dirt_amt);
  }
  seg(S->L.o_pcg, S->L.o_logic);
}

// creation (init=1): random.seed(py_seed), Factory.__init__ (floor list, OBSBuilder shuffle); then reset.
// The first observation is rendered by k_obs afterwards.
#ifndef MFG_OBS_UNIT  // host-unit kernel (not compiled in the render units)
template <int NW>
static __global__ void __launch_bounds__(MFG_WPB * 64) k_reset(const MfgDevSpec* S_, uint8_t* state, long long B,
                                                        const uint8_t* mask, int init, unsigned long long seed_base) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  SpecP S = (SpecP)S_;
  const int wid = uni(threadIdx.x >> 6);  // wave-uniform: slice and record addresses become scalar
  const long long env = (long long)blockIdx.x * (blockDim.x >> 6) + wid;
  if (env >= B) return;
  if (mask && !mask[env]) return;
  Env e;
  env_full(S, smem + (size_t)wid * S->lds_full, e, env);
  uint8_t* rec = state + (size_t)env * S->L.size;
  if (init & MFG_INIT_CREATE) {
    if (init & MFG_INIT_KEEP_MT) {
      // MT19937 state imported by the caller (e.g. Python's global `random` state): keep it, zero the rest
      rec_copy(e.lds, rec, S->L.size, e.lane);
      wave_sync();
      const int mt_idx = e.H(H_MT_IDX);
      const int w0 = S->L.o_mt >> 2, w1 = (S->L.o_mt >> 2) + 624;
      for (int i = e.lane; i < (S->L.size >> 2); i += MFG_WAVE)
        if (i < w0 || i >= w1) ((int*)e.lds)[i] = 0;
      wave_sync();
      e.setH(H_MT_IDX, mt_idx);
    } else {
      for (int i = e.lane; i < (S->L.size >> 2); i += MFG_WAVE) ((int*)e.lds)[i] = 0;
      wave_sync();
      const unsigned long long py_seed = seed_base + (unsigned long long)env;
      uint32_t key[2] = {(uint32_t)py_seed, (uint32_t)(py_seed >> 32)};
      mt_seed(e, key, key[1] ? 2 : 1);
    }
    for (int i = e.lane; i < S->nf; i += MFG_WAVE) e.perm()[i] = (uint16_t)S->floor_init[i];
    if (e.lane == 0) {
      e.pcg()[0] = S->pcg_init_hi; e.pcg()[1] = S->pcg_init_lo;
      e.pcg()[2] = S->pcg_inc_hi;  e.pcg()[3] = S->pcg_inc_lo;
    }
#pragma unroll
    for (int h = 0; h < NW; h++)
      if (h * MFG_WAVE + e.lane < S->nd) e.door()[h * MFG_WAVE + e.lane] = DW_PRESENT;
    for (int r = 0; r < S->s.n_rules; r++) {
      const CS mfg_rule& ru = S->s.rules[r];
      if (e.lane == 0 && ru.op == MFG_RULE_RESPAWN_ITEMS) e.rctr()[r] = ru.i[1];
      if (e.lane == 0 && ru.op == MFG_RULE_RESPAWN_DIRT) e.rctr()[r] = ru.i[0];
    }
    e.setH(H_EPISODE, -1);
    wave_sync();
    floor_shuffle(e);  // OBSBuilder.__init__: `for pos in state.entities.floorlist` (observation_builder.py:57)
  } else {
    rec_copy(e.lds, rec, S->L.size, e.lane);
    wave_sync();
  }
  if (!(init & MFG_INIT_NO_RESET)) {
    env_reset<NW>(e, e.scratch);
    e.setH(H_OBS_INIT, 1);  // the reference renders right after every reset
  }
  e.setH(H_DONE, 0);
  e.setH(H_DIRT_TOUCH, 0);
  wave_sync();
  rec_copy(rec, e.lds, S->L.size, e.lane);
}
#endif

// One env-step of every env (no reset, no render). FULL: the spec consumes the floor order inside a
// step (S->step_rng), so the whole record incl. MT/perm is staged; otherwise only the lean prefix.
#ifndef MFG_OBS_UNIT  // host-unit kernel (not compiled in the render units)
template <bool FULL, bool MAINT, int SEL, int NW>
static __global__ void __launch_bounds__(MFG_WPB * 64) MFG_WPE_LOGIC(FULL || MAINT ? 1 : 8) k_logic(const MfgDevSpec* S_, uint8_t* state, long long B,
                                                        const int32_t* actions, unsigned philox_seed,
                                                        unsigned env_base, long long step, double* reward,
                                                        uint8_t* done, uint8_t* ev_act, uint8_t* ev_watch,
                                                        int32_t* ev_misc, int auto_reset, int rd_slot) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  SpecP S = (SpecP)S_;
  const int wid = threadIdx.x >> 6;  // (a uniform wid here measured slower: 0.319 vs 0.298 ms at C3)
  const long long env = (long long)blockIdx.x * (blockDim.x >> 6) + wid;
  if (env >= B) return;
  // SEL (specs whose only in-step RNG consumer is RespawnDirt): 1 = the envs where no spawn fires this step (the
  // lean k_logic<false, false, 1>, launched first), 2 = the envs where one fires (k_logic<true, false, 2>, after
  // it); 0 = every env. A spawn fires exactly when its rule counter is 0 at the start of the step
  // (clean_up/rules.py:49-59). The first launch has already stepped (and counted down) the other envs when the
  // second runs, so it marks the envs it leaves in rd_flag (2), which the second takes and overwrites.
  if constexpr (SEL == 1) {
    const uint8_t* grec = state + (size_t)env * S->L.size;
    const int* rc = (const int*)(grec + S->L.o_rule_ctr);
    bool fire = false;
    for (uint32_t m = S->respawn_mask; m; m &= m - 1) fire |= uni(rc[__ffs(m) - 1]) == 0;
    if constexpr (MAINT) {
      // a maintainer needs the floor order / MT / BFS only when its path is used up at its tick (maint_tick:
      // a new route, maintenance/entitites.py get_move_action); nothing changes its path before that tick
      const int nk = uni(((const int*)(grec + S->L.o_hdr))[H_N_MAINTS]);
      for (int k = 0; k < nk; k++) {
        const int* st = (const int*)(grec + S->L.o_mstate) + k * S->mstate_ints;
        fire |= uni(st[MS_PATH_HEAD]) >= uni(st[MS_PATH_N]);
      }
    }
    if (fire) {
      if (lane_id() == 0) S->rd_flag[env] = 2;
      return;
    }
  } else if constexpr (SEL == 2) {
    if (uni((int)S->rd_flag[env]) != 2) return;
  }
  Env e;
  // MAINT, SEL 1: the step prefix, then the maintainer states [o_mstate, o_mpath) (16-B rounded) right after it
  // instead of at their record offset (mdelta), then the count scratch: no MT, permutation or BFS scratch. A step of
  // these envs reads one cell of each maintainer's path (the one it advances to), in place in HBM: staging the whole
  // paths (C5: 4 x 1,000 cells) was most of this launch's traffic (round 6)
  constexpr bool lm = MAINT && SEL == 1;
  const int ms0 = S->L.o_mstate & ~15, mlen = lm ? ((S->L.o_mpath + 15) & ~15) - ms0 : 0;
  uint8_t* slice = smem + (size_t)wid * (lm ? S->L.o_logic + mlen + 4 * MFG_WAVE * NW : S->lds_logic);
  constexpr bool full = FULL && !lm;
  if (full) {
    env_full(S, slice, e, env);
  } else {
    e.S = S; e.lds = slice; e.scratch = (int*)(slice + S->L.o_logic + mlen); e.stab = nullptr; e.cmap = nullptr;
    e.bfs = nullptr; e.hdrp = (int*)(slice + S->L.o_hdr); e.lane = lane_id();
    if (lm) {
      e.mdelta = S->L.o_logic - ms0;
      e.gpath = (const uint16_t*)(state + (size_t)env * S->L.size + S->L.o_mpath);
    }
  }
  uint8_t* rec = state + (size_t)env * S->L.size;
  // FULL without maintainers: a RespawnDirt rule is the only in-step reader of the MT state and the floor order, and
  // it spawns exactly when its counter is 0 at the start of the step (clean_up/rules.py:49-59; nothing else changes
  // the counter before its tick). So only the lean prefix is staged, and the MT/perm tail only in the envs where a
  // spawn fires (k_replay_sel paid their earlier debt): C4 ~1/16 of the envs per step.
  constexpr bool lazy = FULL && !MAINT;
  const int bytes = full && !lazy ? S->L.size : S->L.o_logic;
  // lean records of <= 1 KiB: each lane keeps its 16-B chunk and writes it back only if the step changed it
  // (most of the record is per-episode constant: frozen origins, ids, counters of idle rules)
  const bool one_pass = (!full || lazy) && (bytes >> 4) <= MFG_WAVE;  // (lm: full is false)
  uint4 orig = make_uint4(0, 0, 0, 0);
  if (one_pass && e.lane < (bytes >> 4)) orig = ((const uint4*)rec)[e.lane];
  // longer lean prefixes with dirt: only the live piles' slots (C2 / C4 / C5: 256 / 128 / 384 slots of 16 B). A lean
  // step never appends a pile (only RespawnDirt does, in the FULL instantiations), so the count it starts with bounds
  // every slot it reads or writes.
  // (MAINT, SEL 1 too: its envs have no dirt spawn this step, so no pile is appended either)
  const bool trim = MFG_LOGIC_TRIM && (!FULL || lm) && !one_pass && S->dirt_cap;
  const int nd0 = trim ? min(uni(((const int*)(rec + S->L.o_hdr))[H_N_DIRT]), S->dirt_cap) : 0;
  // the actions (a buffer load or Philox) while the record load is in flight
  const int A = S->A;
  int my_act[NW];
#pragma unroll
  for (int h = 0; h < NW; h++) {
    const int a = h * MFG_WAVE + e.lane;
    my_act[h] = 0;
    if (a < A) {
      if (actions) {
        my_act[h] = actions[(size_t)env * A + a];
      } else {
        const uint32_t u = philox_u32(philox_seed, env_base + (uint32_t)env, (uint32_t)step, (uint32_t)a);
        my_act[h] = (int)(((uint64_t)u * (uint64_t)S->s.n_actions[a]) >> 32);
      }
    }
  }
  if (one_pass) {
    if (e.lane < (bytes >> 4)) ((uint4*)e.lds)[e.lane] = orig;
  } else if (trim) {
    prefix_copy(e.lds, rec, S, nd0, e.lane);
  } else {
    rec_copy(e.lds, rec, bytes, e.lane);
  }
  wave_sync();
  if constexpr (lm) {
    rec_copy(e.lds + S->L.o_logic, rec + ms0, mlen, e.lane);
    wave_sync();
  }
  // the RNG tail [o_mt, o_mstate) rounded to 16 B (o_mt is 16-B aligned; the rounding stays inside the record)
  const int o_tail = S->L.o_mt, n_tail = (S->L.o_mstate - S->L.o_mt + 15) & ~15;
  bool rng_tail = false;
  if constexpr (lazy) {
    for (uint32_t m = S->respawn_mask; m; m &= m - 1) rng_tail |= uni(e.rctr()[__ffs(m) - 1]) == 0;
    if (rng_tail) {
      rec_copy(e.lds + o_tail, rec + o_tail, n_tail, e.lane);
      wave_sync();
    }
  }
  StepOut<NW> o;
  env_step<FULL, MAINT, NW>(e, my_act, o, e.scratch);
  write_step_outputs(e, o, (size_t)env, reward, done, ev_act, ev_watch, ev_misc);
  if (e.lane == 0) S->rd_flag[env] = (o.done && auto_reset) ? 1 : 0;
  if (o.done && auto_reset) {
    e.setH(H_DONE, 1);
    // append to this step's done list (k_resetdone walks it instead of one wave per env)
    int32_t* lst = S->rd_list + (size_t)rd_slot * (size_t)(B + 2);
    if (e.lane == 0) lst[2 + atomicAdd(&lst[0], 1)] = (int32_t)env;
  }
  // the next step's list is empty ([0] count, [1] k_replay_done's taken counter): its last reader (the previous
  // step's k_resetdone) has finished
  if (blockIdx.x == 0 && threadIdx.x < 2) S->rd_list[(size_t)(rd_slot ^ 1) * (size_t)(B + 2) + threadIdx.x] = 0;
  wave_sync();
  // most lean steps touch no dirt pile (C5: ~6 of its ~8 KB prefix are the live piles' slots): with trim those slots
  // go back only when the step changed one (the flag is step-local: cleared in every record written back)
  const bool dirt_w = e.H(H_DIRT_TOUCH) != 0;
  wave_sync();
  e.setH(H_DIRT_TOUCH, 0);
  wave_sync();
  if (one_pass) {
    if (e.lane < (bytes >> 4)) {
      const uint4 v = ((const uint4*)e.lds)[e.lane];
      if (v.x != orig.x || v.y != orig.y || v.z != orig.z || v.w != orig.w) ((uint4*)rec)[e.lane] = v;
    }
  } else if (trim) {
    prefix_copy(rec, e.lds, S, nd0, e.lane, dirt_w);
  } else {
    rec_copy(rec, e.lds, bytes, e.lane);
  }
  if (lazy && rng_tail) rec_copy(rec + o_tail, e.lds + o_tail, n_tail, e.lane);
  // (lm: only the maintainer states go back; their paths are read-only here, since a maintainer whose path is used
  // up re-routes in the SEL 2 launch, and C5's 4 x 1,000-cell paths were most of k_logic's writes)
  if constexpr (lm) rec_copy(rec + ms0, e.lds + S->L.o_logic, mlen, e.lane);
}
#endif

// Auto-reset of the envs k_logic flagged (H_DONE) in this step's done list: pays the shuffle debt, then
// Factory.reset(). A fixed grid of waves strides over the list (count <= B, every wave exits), so a step
// with few episode ends costs a few waves instead of one wave per env.
#ifndef MFG_OBS_UNIT  // host-unit kernel (not compiled in the render units)
template <int NW>
static __global__ void __launch_bounds__(MFG_WPB * 64) __attribute__((amdgpu_waves_per_eu(4)))
k_resetdone(const MfgDevSpec* S_, uint8_t* state, long long B, int rd_slot) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  SpecP S = (SpecP)S_;
  const int wid = uni(threadIdx.x >> 6);  // wave-uniform: slice and record addresses become scalar
  const int32_t* lst = S->rd_list + (size_t)rd_slot * (size_t)(B + 2);
  const long long n = min((long long)uni(lst[0]), B);
  const long long nw = (long long)gridDim.x * (blockDim.x >> 6);
  for (long long q = (long long)blockIdx.x * (blockDim.x >> 6) + wid; q < n; q += nw) {
    const long long env = uni(lst[2 + q]);
    if (env < 0 || env >= B) continue;
    uint8_t* rec = state + (size_t)env * S->L.size;
    if (uni(((const int*)(rec + S->L.o_hdr))[H_DONE]) == 0) continue;
    Env e;
    env_full(S, smem + (size_t)wid * S->lds_full, e, env);
    rec_copy(e.lds, rec, S->L.size, e.lane);
    wave_sync();
    env_reset<NW>(e, e.scratch);
    e.setH(H_DONE, 0);
    e.setH(H_DIRT_TOUCH, 0);
    wave_sync();
    rec_copy(rec, e.lds, S->L.size, e.lane);
    wave_sync();
  }
}
#endif

// Observation render of every env into obs[env] (read-only on the state). MM: the spec has machines or
// maintainers (their tags, identifiers and dedupe); compiled out otherwise to keep the VGPR budget.
// One env's render (observation_builder.py:138-235) in its LDS slice.
template <int MAXPTS, typename OT, bool MM, int PK, bool DIRT, bool MW = false>
__device__ __forceinline__ void obs_env(SpecP S, uint8_t* slice, const uint8_t* state, long long env, OT* obs,
                                        ObsPacked pk, int wv = 0, int nwv = 1, int slot = 0) {
  // slice: [lean record][cell map][pairs] (+ per-wave tables, build_obs)
  Env e;
  e.S = S; e.lds = slice; e.stab = nullptr;
  e.cmap = slice + S->L.o_mt;
  e.scratch = (int*)(slice + S->L.o_mt + (MM ? S->map_bytes : S->map_bytes8));
  e.hdrp = (int*)(slice + S->L.o_hdr);
  e.lane = lane_id();
  const uint8_t* rec = state + (size_t)env * S->L.size;
  if constexpr (MW) {
    const int n16 = S->L.o_mt >> 4;
    for (int i = wv * MFG_WAVE + e.lane; i < n16; i += MFG_WAVE * nwv) ((uint4*)e.lds)[i] = ((const uint4*)rec)[i];
  } else {
    rec_copy(e.lds, rec, S->L.o_mt, e.lane);
  }
  mw_sync<MW>();
  int* pg = S->pair_pool ? S->pair_pool + (size_t)env * 3 * (S->max_pairs - S->pairs_lds) : nullptr;
  if constexpr (PK) {  // this env's rows of the packed buffers
    const size_t ea = (size_t)env * S->A;
    pk.idx = pk.idx ? pk.idx + ea * pk.cap : nullptr;
    pk.val = pk.val ? pk.val + ea * pk.cap : nullptr;
    pk.cnt = pk.cnt ? pk.cnt + ea : nullptr;
    pk.emb = pk.emb ? pk.emb + ea * pk.E : nullptr;
    build_obs<MAXPTS, OT, MM, PK, DIRT, MW>(e, nullptr, pg, pk, wv, nwv, slot);
  } else {
    build_obs<MAXPTS, OT, MM, PK, DIRT, MW>(e, obs + (size_t)env * S->A * S->obs_agent_stride, pg, pk, wv, nwv, slot);
  }
  // k_obs reads only [0, o_mt) of the record and stores only this word: the replay of the same call may run beside it
  // on the engine's second stream and writes H_DEBT / H_MT_IDX (single words) and [o_mt, o_perm + 2 nf) (replay_env)
  if ((!MW || wv == 0) && e.lane == 0 && e.hdrp[H_OVERFLOW])
    ((int*)(state + (size_t)env * S->L.size + S->L.o_hdr))[H_OVERFLOW] = 1;
  if constexpr (MW) __syncthreads();  // the shared tables are free for the workgroup's next env
}

// Render of every env (skip: envs k_logic put on this step's done list, rendered by k_obs_list after their reset
// on the engine's second stream; null = none). With auto-reset, mfg_step renders the envs that did not finish
// on the caller's stream while the finished ones are reset and rendered beside it.
template <int MAXPTS, typename OT, bool MM, int PK, bool DIRT>
static __global__ void __launch_bounds__(MFG_WPB * 64) __attribute__((amdgpu_waves_per_eu(MAXPTS <= 8 ? 7 : 1))) k_obs(const MfgDevSpec* S_, const uint8_t* state, long long B,
                                                      OT* obs, ObsPacked pk, const uint8_t* skip) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  SpecP S = (SpecP)S_;
  const int wid = uni(threadIdx.x >> 6);  // wave-uniform: slice and record addresses become scalar
  const long long env = (long long)blockIdx.x * (blockDim.x >> 6) + wid;
  if (env >= B) return;
  if (skip && skip[env]) return;
  obs_env<MAXPTS, OT, MM, PK, DIRT>(S, smem + (size_t)wid * S->lds_obs, state, env, obs, pk);
}
// Multi-wave render: one env per workgroup of nwv waves (specs whose per-env render slice is large, C5: a
// 128 x 128 u16 cell map; the waves share it and split the agents)
template <int MAXPTS, typename OT, bool MM, int PK, bool DIRT>
static __global__ void __launch_bounds__(8 * 64) k_obs_mw(const MfgDevSpec* S_, const uint8_t* state, long long B,
                                                           OT* obs, ObsPacked pk, const uint8_t* skip) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  SpecP S = (SpecP)S_;
  const long long env = blockIdx.x;
  if (env >= B || (skip && skip[env])) return;  // uniform over the workgroup
  obs_env<MAXPTS, OT, MM, PK, DIRT, true>(S, smem, state, env, obs, pk, uni(threadIdx.x >> 6), blockDim.x >> 6);
}
template <int MAXPTS, typename OT, bool MM, int PK, bool DIRT>
static __global__ void __launch_bounds__(8 * 64) k_obs_mw_list(const MfgDevSpec* S_, const uint8_t* state,
                                                                long long B, OT* obs, ObsPacked pk,
                                                                const int32_t* list) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  SpecP S = (SpecP)S_;
  const long long n = min((long long)uni(list[0]), B);
  for (long long q = blockIdx.x; q < n; q += gridDim.x) {
    const long long env = uni(list[2 + q]);
    if (env >= 0 && env < B)
      obs_env<MAXPTS, OT, MM, PK, DIRT, true>(S, smem, state, env, obs, pk, uni(threadIdx.x >> 6), blockDim.x >> 6);
  }
}
// Long-ray render (rays of 65..255 points: pomdp_r 32..126, full observability on levels with min(H, W) 64..254): a
// resident grid of single-wave workgroups strides over every env (skip: envs left to the list render) or over a done
// list; workgroup g owns HBM pool slot g for its per-agent tables (build_obs, LR), its LDS slice holds the lean record,
// the cell map and the identifier pairs.
// The done-list render (list != null, the engine's second stream) and the render of the other envs (the caller's
// stream) may run at the same time: the list render owns slots [obs_slots, 2 obs_slots), the other one [0, obs_slots).
template <typename OT, bool MM, int PK, bool DIRT>
static __global__ void __launch_bounds__(MFG_WAVE) k_obs_lr(const MfgDevSpec* S_, const uint8_t* state, long long B,
                                                            OT* obs, ObsPacked pk, const uint8_t* skip,
                                                            const int32_t* list) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  SpecP S = (SpecP)S_;
  const long long n = list ? min((long long)uni(list[0]), B) : B;
  const int slot = (int)blockIdx.x + (list ? S->obs_slots : 0);  // gridDim.x <= obs_slots (launch_obs_t)
  for (long long q = blockIdx.x; q < n; q += gridDim.x) {
    const long long env = list ? (long long)uni(list[2 + q]) : q;
    if (env < 0 || env >= B || (!list && skip && skip[env])) continue;
    obs_env<0, OT, MM, PK, DIRT>(S, smem, state, env, obs, pk, 0, 1, slot);
  }
}
// Render of the envs of a done list (rd_list row: [0] = count, [2..] = envs): a resident grid strides over it.
template <int MAXPTS, typename OT, bool MM, int PK, bool DIRT>
static __global__ void __launch_bounds__(MFG_WPB * 64) k_obs_list(const MfgDevSpec* S_, const uint8_t* state, long long B,
                                                           OT* obs, ObsPacked pk, const int32_t* list) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  SpecP S = (SpecP)S_;
  const int wid = uni(threadIdx.x >> 6);
  const long long n = min((long long)uni(list[0]), B);
  const long long nw = (long long)gridDim.x * (blockDim.x >> 6);
  for (long long q = (long long)blockIdx.x * (blockDim.x >> 6) + wid; q < n; q += nw) {
    const long long env = uni(list[2 + q]);
    if (env >= 0 && env < B) obs_env<MAXPTS, OT, MM, PK, DIRT>(S, smem + (size_t)wid * S->lds_obs, state, env, obs, pk);
  }
}

// Pay one env's pending floor-shuffle debt in a k_replay-sized LDS slice. Touches only the header, MT state
// and floor permutation of the record, so it runs at high occupancy.
__device__ __forceinline__ void replay_env(SpecP S, uint8_t* slice, uint8_t* rec) {
  const int debt = ((const int*)(rec + S->L.o_hdr))[H_DEBT];
  if (debt == 0) return;
  // LDS slice laid out like the record prefix so Env accessors work: [hdr .. o_mt .. o_perm end]
  Env e;
  e.S = S;
  e.lds = slice - S->L.o_mt + 4 * RP_HDR_N;
  e.lane = lane_id();
  e.scratch = (int*)(slice + S->replay_sink_off);
  e.cmap = nullptr;
  e.stab = (uint32_t*)(slice + S->replay_stab_off);
  e.hdrp = (int*)slice;
  int* hdr = e.hdr();
  const int n16 = S->replay_mtperm >> 4;  // MT + u16 perm image of the record, 16 B units
  if (e.lane < RP_HDR_N) hdr[e.lane] = ((const int*)(rec + S->L.o_hdr))[e.lane];
  {
    const uint4* src = (const uint4*)(rec + S->L.o_mt);
    uint4* dst = (uint4*)(e.lds + S->L.o_mt);
    for (int i = e.lane; i < n16; i += MFG_WAVE) dst[i] = src[i];
  }
  for (int i = e.lane; i < S->replay_stab_n; i += MFG_WAVE) e.stab[i] = 0u;
  wave_sync();
  if (S->xchg_ordered) {
    const int d = e.H(H_DEBT);
    for (int k = 0; k < d; k++) replay_shuffle(e, e.perm());
    e.setH(H_DEBT, 0);
    wave_sync();
  } else {
    pay_debt(e);
  }
  {
    const uint4* src = (const uint4*)(e.lds + S->L.o_mt);
    uint4* dst = (uint4*)(rec + S->L.o_mt);
    for (int i = e.lane; i < n16; i += MFG_WAVE) dst[i] = src[i];
  }
  // Word-granular header write-back, on purpose: in split mode (mfg_step, replay beside the last k_obs on the second
  // stream) k_obs may read this record's header and store its H_OVERFLOW word at the same time. k_obs never reads
  // H_DEBT / H_MT_IDX or anything at or past o_mt, and these two single-word stores never touch H_OVERFLOW; a vector
  // store of the header here would race with it.
  static_assert(H_OVERFLOW != H_DEBT && H_OVERFLOW != H_MT_IDX, "replay header words must not cover H_OVERFLOW");
  if (e.lane == 0) {
    ((int*)(rec + S->L.o_hdr))[H_DEBT] = 0;
    ((int*)(rec + S->L.o_hdr))[H_MT_IDX] = hdr[H_MT_IDX];
  }
  wave_sync();
}

// Pay every env's pending floor-shuffle debt (once per mfg_step call). order (optional): the envs in
// launch order, longest debt first (k_rp_count/k_rp_scan/k_rp_place), so the launch's drain runs short debts.
#ifndef MFG_OBS_UNIT  // host-unit kernel (not compiled in the render units)
static __global__ void __launch_bounds__(MFG_WPB * 64) k_replay(const MfgDevSpec* S_, uint8_t* state, long long B,
                                                         const int* order) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  SpecP S = (SpecP)S_;
  const int wid = uni(threadIdx.x >> 6);  // wave-uniform: the slice addresses become scalar
  long long env = (long long)blockIdx.x * (blockDim.x >> 6) + wid;
  if (env >= B) return;
  if (order) env = uni(order[env]);
  replay_env(S, smem + (size_t)wid * S->lds_replay_per_wave, state + (size_t)env * S->L.size);
}
#endif

// Two-wave replay of one env (workgroup of 128 threads; slice = the 1-wave slice + the chunk ring): wave 0
// produces the draws, wave 1 applies the swap blocks (rp2_produce / rp2_consume). Needs the ordered exchange.
__device__ void replay_env2(SpecP S, uint8_t* slice, uint8_t* rec) {
  const int wv = uni(threadIdx.x >> 6);
  const int debt = uni(((const int*)(rec + S->L.o_hdr))[H_DEBT]);
  if (debt == 0) return;  // uniform over the workgroup
  Env e;
  e.S = S;
  e.lds = slice - S->L.o_mt + 4 * RP_HDR_N;
  e.lane = lane_id();
  e.scratch = (int*)(slice + S->replay_sink_off);
  e.cmap = nullptr;
  e.stab = (uint32_t*)(slice + S->replay_stab_off);
  e.hdrp = (int*)slice;
  uint8_t* ring = slice + S->lds_replay_per_wave;
  int* ctl = (int*)(ring + 2 * RP2_R * RP2_REC);  // [0], [1]: chunks in each half; [2]: the producer's last phase
  const int t = wv * MFG_WAVE + e.lane;
  const int n16 = S->replay_mtperm >> 4;
  if (t < RP_HDR_N) e.hdrp[t] = ((const int*)(rec + S->L.o_hdr))[t];
  {
    const uint4* src = (const uint4*)(rec + S->L.o_mt);
    uint4* dst = (uint4*)(e.lds + S->L.o_mt);
    for (int i = t; i < n16; i += 2 * MFG_WAVE) dst[i] = src[i];
  }
  for (int i = t; i < S->replay_stab_n; i += 2 * MFG_WAVE) e.stab[i] = 0u;
  if (t == 0) ctl[2] = -1;
  __syncthreads();
  const int hi = S->nf - 1;
  Rp2Prod st;
  st.s = 0;
  st.icur = hi;
  st.idx = e.H(H_MT_IDX);
  st.yw = (wv == 0 && st.idx <= 560) ? e.mt()[st.idx + e.lane] : 0u;
  uint32_t ctr = 0;
  for (int phase = 0;; phase++) {
    uint8_t* half = ring + (phase & 1) * RP2_R * RP2_REC;
    if (wv == 0) {
      if (st.s < debt) {
        if (S->replay_top14) rp2_produce<true>(e, half, &ctl[phase & 1], st, debt, hi);
        else rp2_produce<false>(e, half, &ctl[phase & 1], st, debt, hi);
        if (st.s >= debt && e.lane == 0) ctl[2] = phase;
      }
    } else if (phase > 0) {
      const uint8_t* prev = ring + ((phase - 1) & 1) * RP2_R * RP2_REC;
      rp2_consume(e, prev, uni(ctl[(phase - 1) & 1]), ctr);
    }
    __syncthreads();
    const int last = uni(ctl[2]);
    if (last >= 0 && phase > last) break;  // the consumer has applied the producer's last half
  }
  if (wv == 0) {
    int idx = st.idx;
    if (idx > 624) {  // words of the next state were consumed: make the state canonical (CPython's mti)
      mt_twist(e);
      idx -= 624;
    }
    if (e.lane == 0) {
      ((int*)(rec + S->L.o_hdr))[H_DEBT] = 0;
      ((int*)(rec + S->L.o_hdr))[H_MT_IDX] = idx;
    }
  }
  __syncthreads();
  {
    const uint4* src = (const uint4*)(e.lds + S->L.o_mt);
    uint4* dst = (uint4*)(rec + S->L.o_mt);
    for (int i = t; i < n16; i += 2 * MFG_WAVE) dst[i] = src[i];
  }
}
#ifndef MFG_OBS_UNIT
static __global__ void __launch_bounds__(2 * MFG_WAVE) k_replay2(const MfgDevSpec* S_, uint8_t* state, long long B,
                                                                 const int* order) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  SpecP S = (SpecP)S_;
  long long env = blockIdx.x;
  if (env >= B) return;
  if (order) env = uni(order[env]);
  replay_env2(S, smem, state + (size_t)env * S->L.size);
}
#endif

// The debt of the envs whose RespawnDirt rule fires in the coming step (its counter is 0: clean_up/rules.py:49-59
// spawns from the floor order), paid at k_replay's occupancy before k_logic<FULL> reaches the spawn; k_logic then
// pays inline only the debt of that step's own moves (C4: ~1/16 of the envs per step carry up to K steps of debt).
#ifndef MFG_OBS_UNIT  // host-unit kernel (not compiled in the render units)
static __global__ void __launch_bounds__(64) k_replay_sel(const MfgDevSpec* S_, uint8_t* state, long long B) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  SpecP S = (SpecP)S_;
  const long long env = blockIdx.x;
  if (env >= B) return;
  uint8_t* rec = state + (size_t)env * S->L.size;
  const int* rc = (const int*)(rec + S->L.o_rule_ctr);
  bool fire = false;
  for (uint32_t m = S->respawn_mask; m; m &= m - 1) fire |= uni(rc[__ffs(m) - 1]) == 0;
  if (!fire) return;
  replay_env(S, smem, rec);
}
#endif

// Replay launch order by debt, longest first (a counting sort over RP_NB debt buckets; envs are
// independent, so the order changes only which waves are left running at the end of the launch).
// Order within a bucket is arbitrary. hist: RP_NB ints, zero on entry to k_rp_count.
#define RP_NB 256
#ifndef MFG_OBS_UNIT  // host-unit kernel (not compiled in the render units)
static __global__ void __launch_bounds__(256) k_rp_count(const MfgDevSpec* S_, const uint8_t* state, long long B,
                                                  int* hist, uint8_t* key) {
  __shared__ int h[RP_NB];
  SpecP S = (SpecP)S_;
  for (int i = threadIdx.x; i < RP_NB; i += blockDim.x) h[i] = 0;
  __syncthreads();
  const long long env = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (env < B) {
    const int d = min(max(((const int*)(state + (size_t)env * S->L.size + S->L.o_hdr))[H_DEBT], 0), 4095);
    // debts < 64 exact, above that 32 buckets per power of two (C3 K=8 debts are ~100, C5's ~1000)
    const int lg = 31 - __clz(d | 1);
    const int q = d < 64 ? d : 64 + (lg - 6) * 32 + ((d >> (lg - 5)) & 31);
    const int b = RP_NB - 1 - q;  // bucket 0: the largest debts
    key[env] = (uint8_t)b;
    atomicAdd(&h[b], 1);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < RP_NB; i += blockDim.x)
    if (h[i]) atomicAdd(&hist[i], h[i]);
}
#endif
#ifndef MFG_OBS_UNIT  // host-unit kernel (not compiled in the render units)
static __global__ void __launch_bounds__(RP_NB) k_rp_scan(int* hist) {  // one block: exclusive scan in place
  __shared__ int s[RP_NB];
  const int t = threadIdx.x;
  const int c = hist[t];
  s[t] = c;
  __syncthreads();
  for (int o = 1; o < RP_NB; o <<= 1) {
    const int v = t >= o ? s[t - o] : 0;
    __syncthreads();
    s[t] += v;
    __syncthreads();
  }
  hist[t] = s[t] - c;
}
#endif
#ifndef MFG_OBS_UNIT  // host-unit kernel (not compiled in the render units)
static __global__ void __launch_bounds__(256) k_rp_place(long long B, int* offs, const uint8_t* key, int* order) {
  __shared__ int h[RP_NB], base[RP_NB];
  for (int i = threadIdx.x; i < RP_NB; i += blockDim.x) h[i] = 0;
  __syncthreads();
  const long long env = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  int b = 0, r = 0;
  if (env < B) {
    b = key[env];
    r = atomicAdd(&h[b], 1);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < RP_NB; i += blockDim.x) base[i] = h[i] ? atomicAdd(&offs[i], h[i]) : 0;
  __syncthreads();
  if (env < B) order[base[b] + r] = (int)env;
}
#endif

// The same for the envs on a step's done list, before k_resetdone resets them: their debt is paid at
// k_replay's occupancy instead of inside the reset kernel's much larger slice. A grid of resident waves
// strides over the list (every wave exits).
#ifndef MFG_OBS_UNIT  // host-unit kernel (not compiled in the render units)
static __global__ void __launch_bounds__(MFG_WPB * 64) k_replay_done(const MfgDevSpec* S_, uint8_t* state, long long B,
                                                              int rd_slot) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  SpecP S = (SpecP)S_;
  const int wid = uni(threadIdx.x >> 6);
  const int32_t* lst = S->rd_list + (size_t)rd_slot * (size_t)(B + 2);
  const long long n = min((long long)uni(lst[0]), B);
  // each wave's first env is its own index; after that the waves take entries nw, nw + 1, ... from a work queue
  // (lst[1] counts the entries taken, k_logic zeroes it with the count): debts differ per env, so a wave takes
  // its next env when it is done instead of a fixed stride. A step with few episode ends touches the counter
  // only from the waves that had an env; every wave exits once its index passes n.
  int* taken = S->rd_list + (size_t)rd_slot * (size_t)(B + 2) + 1;
  const long long nw = (long long)gridDim.x * (blockDim.x >> 6);
  long long q = (long long)blockIdx.x * (blockDim.x >> 6) + wid;
  while (q < n) {
    const long long env = uni(lst[2 + q]);
    if (env >= 0 && env < B)
      replay_env(S, smem + (size_t)wid * S->lds_replay_per_wave, state + (size_t)env * S->L.size);
    int t = 0;
    if (__lane_id() == 0) t = atomicAdd(taken, 1);
    q = nw + rl(t, 0);
  }
}
#endif


// ------------------------------------------------------------------------------------------------
// observation-render launch (instantiated in the mfg_obs_*.hip units, per ray length MP)
// ------------------------------------------------------------------------------------------------
struct ObsLaunch {
  const MfgDevSpec* d_spec;
  uint8_t* d_state;
  long long B;
  bool mm, dirt;     // spec has machines/maintainers; spec has dirt piles
  bool mw;           // multi-wave render (one env per workgroup of W waves, k_obs_mw; ray lengths >= 10 only)
  unsigned grid;     // workgroups
  int W;             // waves per workgroup
  size_t lds;        // dynamic LDS per workgroup
};
// k_obs over every env (list = null; skip: flags of envs left to a list render) or over a done list (a resident
// grid striding over it)
template <int MP, typename OT, int PK>
hipError_t launch_obs_inst(const ObsLaunch& L, OT* obs, const ObsPacked& pk, hipStream_t st, const uint8_t* skip,
                           const int32_t* list);
#define MFG_DEFINE_LAUNCH_OBS                                                                                    \
  template <int MP, typename OT, int PK>                                                                        \
  hipError_t launch_obs_inst(const ObsLaunch& L, OT* obs, const ObsPacked& pk, hipStream_t st,                   \
                             const uint8_t* skip, const int32_t* list) {                                        \
    MFG_OBS_LAUNCH_IF(true, true) else MFG_OBS_LAUNCH_IF(true, false) else MFG_OBS_LAUNCH_IF(false, true)          \
    else MFG_OBS_LAUNCH_IF(false, false)                                                                         \
    return hipGetLastError();                                                                                    \
  }
#define MFG_OBS_LAUNCH_IF(MMV, DV)                                                                               \
  if (L.mm == MMV && L.dirt == DV) {                                                                             \
    bool mw_done = false;                                                                                        \
    if constexpr (MP == 0) {                                                                                     \
      mw_done = true;                                                                                            \
      hipLaunchKernelGGL((k_obs_lr<OT, MMV, PK, DV>), dim3(L.grid), dim3(64), L.lds, st, L.d_spec, L.d_state,    \
                         L.B, obs, pk, skip, list);                                                              \
    }                                                                                                            \
    if constexpr (MP >= 10) {                                                                                    \
      if (L.mw) {                                                                                                \
        mw_done = true;                                                                                          \
        if (list)                                                                                                \
          hipLaunchKernelGGL((k_obs_mw_list<MP, OT, MMV, PK, DV>), dim3(L.grid), dim3(L.W * 64), L.lds, st,      \
                             L.d_spec, L.d_state, L.B, obs, pk, list);                                           \
        else                                                                                                     \
          hipLaunchKernelGGL((k_obs_mw<MP, OT, MMV, PK, DV>), dim3(L.grid), dim3(L.W * 64), L.lds, st, L.d_spec, \
                             L.d_state, L.B, obs, pk, skip);                                                     \
      }                                                                                                          \
    }                                                                                                            \
    if constexpr (MP != 0) if (!mw_done) {                                                                       \
      if (list)                                                                                                  \
        hipLaunchKernelGGL((k_obs_list<MP, OT, MMV, PK, DV>), dim3(L.grid), dim3(L.W * 64), L.lds, st, L.d_spec, \
                           L.d_state, L.B, obs, pk, list);                                                       \
      else                                                                                                       \
        hipLaunchKernelGGL((k_obs<MP, OT, MMV, PK, DV>), dim3(L.grid), dim3(L.W * 64), L.lds, st, L.d_spec,     \
                           L.d_state, L.B, obs, pk, skip);                                                       \
    }                                                                                                            \
  }
// explicit instantiations of one ray length (the obs modes: packed + fused projection, packed entries only, f64, f32)
#define MFG_INSTANTIATE_OBS(MP)                                                                                  \
  template hipError_t launch_obs_inst<MP, float, 2>(const ObsLaunch&, float*, const ObsPacked&, hipStream_t,      \
                                                    const uint8_t*, const int32_t*);                             \
  template hipError_t launch_obs_inst<MP, float, 1>(const ObsLaunch&, float*, const ObsPacked&, hipStream_t,      \
                                                    const uint8_t*, const int32_t*);                             \
  template hipError_t launch_obs_inst<MP, double, 0>(const ObsLaunch&, double*, const ObsPacked&, hipStream_t,    \
                                                     const uint8_t*, const int32_t*);                            \
  template hipError_t launch_obs_inst<MP, float, 0>(const ObsLaunch&, float*, const ObsPacked&, hipStream_t,      \
                                                    const uint8_t*, const int32_t*);
