// Gradient reduction body shared by k_reduce_adam (tt_optim.hip) and the
// deferred late half inside k_l0_fwd (tt_tower.hip).  See tt_optim.hip.
#pragma once
#include "tt_common.h"

namespace tt {

// Data-parallel exchange of the reduced gradient (EX instance; all threads of
// the block call it, owner lanes carry an element).  TT_AR_PUSH: the
// flag-in-data words of tt_common.h (ll_publish / ll_gather_sums), one
// barrier.  TT_AR_PULL: the one-shot protocol of
// tt_comm.hip (k_ar_adam) per reduction block: publish this block's sums into
// this rank's slot[t & 1], signal flag[rank][block] = t on every peer, wait
// (bounded) for every peer's flag, then the mean in rank order -- this rank's
// own term from the register, the same bits its slot holds, so every rank
// computes bitwise the same mean.  World 1: nothing to exchange.  Returns
// false (block-uniform) when the exchange is off (sticky err) or timed out:
// the caller then leaves this block's parameters and Adam state untouched.
// Slot reuse: rank r rewrites slot[t & 1] at step t + 2, after its step-t+1
// block saw every peer's step-t+1 flag, which the peer wrote in a launch that
// started after its step-t launch (the one reading slot[t & 1]) ended.
__device__ __forceinline__ bool reduce_exchange(const RedExchange& X, int64_t t, bool owner, int64_t e, float& g,
                                                int* ok_s) {
  if (*ok_s == 0) return false;
  if (X.world == 1) return true;
  if (X.protocol == TT_AR_PUSH) {  // this element's word into every peer, then poll the own region
    const int64_t par = t & 1;
    const uint32_t ep = (uint32_t)t;
    bool fine = true;
    if (owner) {
      ll_publish(X.ll, X.world, X.rank, X.slot_stride, par, e, g, ep);
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
      const bool live = true;
      float s = 0.f;
      if (X.world <= 2)
        fine = ll_gather_sums<2, 1>(X.ll[X.rank], X.world, X.rank, X.slot_stride, par, &e, &live, &g, ep, t0,
                                    X.wait_ticks, &s);
      else if (X.world <= 4)
        fine = ll_gather_sums<4, 1>(X.ll[X.rank], X.world, X.rank, X.slot_stride, par, &e, &live, &g, ep, t0,
                                    X.wait_ticks, &s);
      else  // (the host allows the push protocol up to TT_AR_PUSH_MAX_RANKS = 8)
        fine = ll_gather_sums<8, 1>(X.ll[X.rank], X.world, X.rank, X.slot_stride, par, &e, &live, &g, ep, t0,
                                    X.wait_ticks, &s);
      if (fine) g = s * (1.0f / (float)X.world);
    }
    if (!fine) *ok_s = 0;  // (every writer stores 0)
    __syncthreads();
    if (*ok_s == 0) {  // block-uniform: this block's parameters stay untouched
      if (threadIdx.x == 0) atomicAdd(X.err, 1);
      return false;
    }
    return true;
  }
  const uint64_t epoch = (uint64_t)t;
  const int b = blockIdx.x, q = threadIdx.x;
  const int64_t par = (t & 1) ? X.slot_stride : 0;
  if (owner) __hip_atomic_store(X.slot[X.rank] + par + e, g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  // every wave's slot stores performed before the barrier that precedes the
  // flags (explicit wait: the fence's own may be dropped, tt_comm.hip)
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (q < X.world && q != X.rank) {
    __hip_atomic_store(X.flags[q] + (int64_t)X.rank * X.blocks + b, epoch, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
    const uint64_t* f = X.flags[X.rank] + (int64_t)q * X.blocks + b;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) < epoch) {
      if (__builtin_amdgcn_s_memrealtime() - t0 > X.wait_ticks) {
        *ok_s = 0;
        atomicAdd(X.err, 1);
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
  }
  __syncthreads();
  if (*ok_s == 0) return false;
  if (owner) {  // every peer's load in flight at once (rank_order_sum), same adds as a rank loop
    const int64_t off = par + e;
    float s;
    if (X.world <= 2)
      s = rank_order_sum<2>(X.slot, X.world, X.rank, off, g);
    else if (X.world <= 4)
      s = rank_order_sum<4>(X.slot, X.world, X.rank, off, g);
    else if (X.world <= 8)
      s = rank_order_sum<8>(X.slot, X.world, X.rank, off, g);
    else
      s = rank_order_sum<TT_AR_MAX_RANKS>(X.slot, X.world, X.rank, off, g);
    g = s * (1.0f / (float)X.world);
  }
  return true;
}

// The reduction body for one element block `bid` (RED_E elements x G slab
// groups = the block's threads).  k_reduce_adam runs it at G = G; a
// deferred late half (LATE, tt_train_step with TT_FLAG_DEFER_LATE) runs it at
// G = LATE_G inside the next step's k_l0_fwd or in tt_train_flush.  LDS:
// part [G][RED_E], xpart [4][G][RED_E] floats, *xok_s.
template <class A, int G, bool PRE, bool EX, bool LATE>
__device__ __forceinline__ void reduce_body(const A& a, int bid, float* part, float* xpart, int* xok_ptr) {
  static_assert(NREP % G == 0 || G % NREP == 0, "kinds 2-4: group pg takes replicas pg, pg + G, ... (none when pg >= NREP)");
  static_assert(RED_E % 32 == 0, "kind 3 pairs lanes el and el + 16 of a 32-lane group");
  int& xok_s = *xok_ptr;  // EX: exchange live (no earlier timeout on this rank)
  auto PART = [&](int k, int e_) -> float& { return part[k * RED_E + e_]; };
  auto XPART = [&](int i, int k, int e_) -> float& { return xpart[(i * G + k) * RED_E + e_]; };
  if constexpr (!LATE) TT_STAMP(5, 0);
  // the step first: a later load would make its wait (in-order vmcnt) wait for the slabs
  // (a select of the two addresses: one FLAT load, issued first -- measured
  // 0.2 us faster here than the global load the tower kernels use).  A late
  // half takes step_done (its early half's step): the next step's k_l0_fwd
  // rewrites step_cur meanwhile
  int64_t t;
  if constexpr (LATE) {
    t = a.state->step_done;
    if (*a.late_pending != t + 1) return;  // nothing deferred by the last step (block-uniform)
  } else {
    t = a.state ? a.state->step_cur : a.step_host;
  }
  const int el = threadIdx.x & (RED_E - 1), pg = threadIdx.x / RED_E;
  const int64_t vb = (int64_t)bid * RED_E;
  // this block's segment: the last entry (block order) starting at or
  // before it, from the compact blk0 / blk_seg arrays -- loaded together,
  // compared in SALU (no dependent load per segment)
  int si = -1;
#pragma unroll
  for (int j = 0; j < (int)(sizeof(a.blk0) / sizeof(a.blk0[0])); ++j)
    if (j < a.n_seg && bid >= a.blk0[j]) si = a.blk_seg[j];
  si = __builtin_amdgcn_readfirstlane(si);
  if (si < 0 || vb >= a.seg[si].voff + a.seg[si].vlen) return;  // (whole block: past the last range)
  const Seg& S = a.seg[si];
  const int kind = S.kind;
  const int64_t dv = vb + el - S.voff;
  // kind 5: element of this lane and its slab half
  static_assert(RED_E == 64 || G * RED_UNR >= 256, "kind 5 (lanes el and el + 32) only at RED_E = 64");
  const bool shalf = kind == 5 && (el & 32) != 0;
  const int64_t ei5 = (dv >> 6) * 32 + (el & 31);
  const bool live = kind == 5 ? ei5 < S.len : dv < S.vlen;
  // parameter element of this lane; kind 3: W0 element and which half (P / Q)
  const bool qhalf = kind == 3 && (el & 16) != 0;
  const int wi = kind == 3 ? (int)(dv >> 5) * 16 + (el & 15) : 0;
  const int64_t e = S.off + (kind == 3 ? (int64_t)wi : kind == 5 ? ei5 : dv);
  // the Adam state of this element is loaded up front: its latency overlaps the slab loads
  const bool owner = pg == 0 && live && !qhalf && !shalf;
  const bool adam_here = owner && a.apply_adam;
  float pp = 0.f, pm = 0.f, pv = 0.f;
  if (adam_here) {
    pp = a.p[e];
    pm = a.m[e];
    pv = a.v[e];
  }
  float acc = 0.f;
  // Adam's bias corrections (double pow: a long dependent chain) are computed
  // by the owner lanes between issuing the slab loads and summing them (was:
  // after the barrier, on the critical path; 8.2 -> 7.3 us).  Owner lanes
  // only: the same pow in every wave costs more (11.4 us) than it hides.
  // (The code shape matters: an equivalent lambda form measured 10.1 us.)
  AdamCoef c{};
  bool coef_done = PRE;
  int ch = 0, kx = 0;  // kinds 3, 4: W0 row / column of this element (kind 4: channel)
  if (kind == 0 || kind == 3 || kind == 5) {
    constexpr int UNR = RED_UNR;
    int64_t so = live ? (kind == 5 ? ei5 : dv) : 0;
    if (kind == 3) {  // P[ch][kx] (or Q); group pg also takes replica pg of the fold sums
      ch = wi / S.in;
      kx = wi - ch * S.in;
      if (!live) ch = kx = 0;
      so = (int64_t)ch * 2 * S.kp + (kx >> 4) * 32 + (kx & 15) + (qhalf ? 16 : 0);
      float r0 = 0.f, r1 = 0.f, r2 = 0.f, r3 = 0.f;
#pragma unroll
      for (int q = pg; q < NREP; q += G) {
        const float* fr = S.rep + (int64_t)q * S.rep_stride;
        r0 += fr[ch];
        r1 += fr[H0 + ch];
        r2 += fr[2 * H0 + ch];
        r3 += fr[3 * H0 + kx];
      }
      XPART(0, pg, el) = r0;
      XPART(1, pg, el) = r1;
      XPART(2, pg, el) = r2;
      XPART(3, pg, el) = r3;
    }
    // fixed summation order (deterministic); UNR independent loads in flight,
    // buffer loads off the block-uniform slab base (32-bit lane offsets: half
    // the address registers of 64-bit pointers)
    const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.slab[S.tower] + S.slab_off), (short)0,
                                                      0x7FFFFFFF, 0x00020000);
    const uint32_t o0 = (uint32_t)so * 4u, ldb = (uint32_t)a.slab_ld * 4u;
    auto ldp = [&](int p) { return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, (int)(o0 + (uint32_t)p * ldb), 0, 0)); };
    const int n = S.n_slabs;
    if (kind == 5) {  // this lane's slab half: [0, 128) or [128, n), one round of loads
      const int pb = shalf ? G * UNR : 0, ne = shalf ? n : min(n, G * UNR);
      float x[UNR];
#pragma unroll
      for (int k = 0; k < UNR; ++k) x[k] = ldp(min(pb + pg + k * G, ne - 1));
      if (!PRE && adam_here) c = adam_coef(a.lr, a.b1, a.b2, a.eps, t);
      coef_done = true;
#pragma unroll
      for (int k = 0; k < UNR; ++k) acc += (pb + pg + k * G < ne) ? x[k] : 0.f;
    } else if (n <= G * (UNR / 2)) {
      // few slabs for this block shape (e.g. 128-row tiles at B = 16384 with
      // 16 groups): half the loads, none of them a clamped repeat
      constexpr int U2 = UNR / 2;
      float x[U2];
#pragma unroll
      for (int k = 0; k < U2; ++k) x[k] = ldp(min(pg + k * G, n - 1));
      if (!PRE && adam_here) c = adam_coef(a.lr, a.b1, a.b2, a.eps, t);
      coef_done = true;
#pragma unroll
      for (int k = 0; k < U2; ++k) acc += (pg + k * G < n) ? x[k] : 0.f;
    } else {
      for (int p0 = pg; p0 < n; p0 += G * UNR) {
        float x[UNR];
#pragma unroll
        for (int k = 0; k < UNR; ++k) x[k] = ldp(min(p0 + k * G, n - 1));
        if (!PRE && !coef_done) {
          if (adam_here) c = adam_coef(a.lr, a.b1, a.b2, a.eps, t);
          coef_done = true;
        }
#pragma unroll
        for (int k = 0; k < UNR; ++k) acc += (p0 + k * G < n) ? x[k] : 0.f;
      }
    }
  } else if (kind == 1) {
    if (pg == 0 && live) acc = a.gacc[e];
  } else if (kind == 2) {  // replicas: group pg sums replicas pg, pg + G, ... (fixed order), zeroes them
    if (live) {
#pragma unroll
      for (int q = pg; q < NREP; q += G) {
        float* rp = S.rep + dv + (int64_t)q * S.rep_stride;
        acc += *rp;
        if (!S.keep) *rp = 0.f;
      }
    }
  } else {  // kind 4: b0 of the folded BN0 backward (replica pg of gg0 | sum Zh0)
    ch = live ? (int)dv : 0;
    float r0 = 0.f, r2 = 0.f;
#pragma unroll
    for (int q = pg; q < NREP; q += G) {
      const float* fr = S.rep + (int64_t)q * S.rep_stride;
      r0 += fr[ch];
      r2 += fr[2 * H0 + ch];
    }
    XPART(0, pg, el) = r0;
    XPART(2, pg, el) = r2;
  }
  if (!PRE && !coef_done && adam_here) c = adam_coef(a.lr, a.b1, a.b2, a.eps, t);
  PART(pg, el) = acc;
  // zero the BN moment sums consumed by this step (one element per thread of
  // the leading blocks); fold the loss replicas (block 0)
  {
    int64_t i = (int64_t)bid * (G * RED_E) + threadIdx.x;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      if (i >= 0 && i < a.zero_len[b]) a.zero_buf[b][i] = 0.f;
      i -= a.zero_len[b];
    }
  }
  if (bid == 0) {
    if (!LATE && a.late_pending && a.late_mark && threadIdx.x == 1)  // the step's deferral record
      *a.late_pending = a.late_mark > 0 ? t + 1 : (int64_t)0;
    if (a.lsr && threadIdx.x == 0) {
      float l = 0.f;
      for (int q = 0; q < NREP; ++q) {
        l += a.lsr[q * LSR + 1];
        a.lsr[q * LSR + 1] = 0.f;
      }
      if (a.loss_state) a.loss_state->loss_sum += l;
    }
  }
  if (EX && threadIdx.x == 0) xok_s = __hip_atomic_load(a.x.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0;
  __syncthreads();
  if constexpr (!LATE) TT_STAMP(5, 1);
  if (!EX && !owner) return;
  float gsum = 0.f;
  if (owner) {
#pragma unroll
    for (int k = 0; k < G; ++k) gsum += PART(k, el);
    if (kind == 5) {  // then the second slab half of the same element (fixed order)
#pragma unroll
      for (int k = 0; k < G; ++k) gsum += PART(k, el + 32);
    }
    if (kind == 3 || kind == 4) {
      // dW0 = k0 (P - mb s - mg Q) + db0 c,  db0 = -k0 mg sum Zh0  (k_bwd_mid_fold)
      float gg = 0.f, zs = 0.f;
#pragma unroll 4
      for (int k = 0; k < G; ++k) {
        gg += XPART(0, k, el);
        zs += XPART(2, k, el);
      }
      const float k0 = S.k0[ch], mg = gg * a.inv_b;
      const float db0 = -k0 * mg * zs;  // = sum over rows of dZ0 (BN0 cancels b0: ~0)
      if (kind == 3) {
        float q = 0.f, gb = 0.f, sx = 0.f;
#pragma unroll 4
        for (int k = 0; k < G; ++k) {
          q += PART(k, el + 16);
          gb += XPART(1, k, el);
          sx += XPART(3, k, el);
        }
        gsum = k0 * (gsum - (gb * a.inv_b) * sx - mg * q) + S.xsh[kx] * db0;
      } else {
        gsum = db0;
      }
    }
  }  // owner
  if constexpr (EX) {
    const bool xok = reduce_exchange(a.x, t, owner, e, gsum, &xok_s);
    if (!owner) return;
    if (!xok) {  // failed exchange: p / m / v / grad untouched, but no stale
      if (kind == 1) a.gacc[e] = 0.f;  // embedding-gradient sums carried into a later step
      return;
    }
  }
  a.grad[e] = gsum;
  if (kind == 1) a.gacc[e] = 0.f;
  if (a.apply_adam) {
    if constexpr (PRE) c = a.adam_slots[t & 1].c;
    adam_elem(pp, pm, pv, gsum, c);
    a.p[e] = pp;
    a.m[e] = pm;
    a.v[e] = pv;
    if constexpr (!LATE) TT_STAMP(5, 2);
    if (!LATE && a.state && bid == 0 && el == 0) a.state->step_done = t;
    if constexpr (PRE) {  // a light block caches the next step's coefficients (AdamSlot)
      if (si == a.next_seg && vb == S.voff && el == 0)
        adam_slot_fill(a.adam_slots[(t + 1) & 1], t + 1, a.lr, a.b1, a.b2, a.eps);
    }
  }
}


}  // namespace tt
