// FlashAttention-2 forward for MI355X (gfx950): O = softmax(scale * Q K^T [+ causal mask]) V, LSE.
//
// Algorithm (the reference's compute_attn_1rowblock, csrc/flash_attn/src/flash_fwd_kernel.h:121-583):
// one workgroup per (query block, batch, head); K/V tiles streamed through LDS; online softmax with
// running max / sum; epilogue O /= l, LSE = max * scale + ln(l) (+inf when l == 0 or NaN,
// flash_fwd_kernel.h:509-518); causal mask is top-left aligned (key <= query, softmax.h:143-178).
//
// MI355X mapping (not a translation of the CUDA tiling):
//   * 8 waves x 32 query rows = 256-row query block per workgroup; BN = 64 keys per K/V tile
//     (d > 128: 4 waves, one per SIMD, and 32-key tiles -- FwdTile).
//   * K/V tiles arrive by LDS-DMA (buffer_load ... lds, one 1-KiB piece per wave instruction) three
//     tiles ahead into a 4-deep LDS ring; the buffer descriptor's range check zero-fills rows past
//     seqlen_k and padded head-dim columns, so the kernel never branches on the load side.  One
//     counted s_waitcnt vmcnt + barrier per tile: the tile issued in this step stays in flight, so
//     each DMA has two tiles of compute to land.
//   * "Swapped" QK^T: each wave computes S^T = K . Q^T with v_mfma_f32_32x32x16, so the query sits on
//     the MFMA column (= lane) and every lane holds 32 scores of ONE query row: the row max / sum are
//     in-lane reductions plus one v_permlane32_swap.
//   * O^T = V^T . P^T: the S^T accumulator, converted to bf16/f16 in registers, is directly the B
//     operand of the PV MFMA (no LDS round trip for P); V^T fragments come from the row-major V tile
//     through ds_read_b64_tr_b16.  O^T keeps the query on the lane, so the online-softmax rescale is
//     a per-lane scalar multiply, deferred (wave-uniformly) until some row max of the wave grew by
//     more than 2^8 (P <= 256 meanwhile; exact in the LSE since m_run is the offset actually used).
//   * Software pipeline over the tiles that need no mask (all but the causal diagonal / the ragged
//     last tile): one basic block per tile holds QK^T(n+1) (MFMA), the exp / sum / pack of tile n
//     (VALU) and PV(n) (MFMA), so the matrix pipe has independent work while the softmax runs.
//   * Every LDS address is one of four per-lane bases + an immediate (fa_common.h LdsBases).
//   * Heaviest causal query blocks are dispatched first (1-D grid, head-fastest) to shorten the tail.
//   * Epilogue: v_permlane32_swap pairs column groups so each lane stores 16 bytes of its O row.
//   * Waves 4-7 (the younger half of the workgroup) run at s_setprio 1 for the whole kernel.
#include <algorithm>
#include <stdexcept>
#include <string>

#include "fa_common.h"
#include "fa_dropout.h"
#include "fa_params.h"

namespace fa {

// Tile shape per head dim.  d <= 128: 8 waves x 32 rows, 64-key tiles, two waves per SIMD.
// d in (128, 256]: the O accumulator (D/2 registers) and the Q fragments (D/4) no longer fit two
// waves per SIMD next to the scores, so a workgroup is 4 waves (one per SIMD, 512 registers each)
// and K/V tiles are 32 keys (the 4-deep ring stays at 4 x 2 x 16 KiB at d = 256).
#ifndef FA_FWD_NW64   // dev switch (A/B): waves per workgroup at head dims <= 64
#define FA_FWD_NW64 8
#endif
template <int D> struct FwdTile {
  static constexpr int NW = D <= 64 ? FA_FWD_NW64 : (D <= 128 ? 8 : 4);
  static constexpr int BM = 32 * NW;
  static constexpr int BN = D <= 128 ? 64 : 32;
  static constexpr int MINB = D <= 128 ? 2 : 1;   // __launch_bounds__ blocks per CU (register budget)
};
constexpr int kFwdBufs = 4;   // K ring depth: tiles nb, nb+1 read while nb+2, nb+3 land

// MASKED: the dense additive mask and/or FlashMask are present; such a launch has no fast path (every
// tile takes the per-element general path), and the unmasked instantiations carry no mask code.
// SPLIT (non-causal, unmasked, no dropout, fixed-length; launch_fwd decides): blockIdx.y selects a
// key range, treated as an attention of its own, and the epilogue writes fp32 partials.
template <bool BF16, int D, bool CAUSAL, bool DROPOUT, bool MASKED, bool SPLIT = false>
__global__ void __launch_bounds__(FwdTile<D>::NW * 64, FwdTile<D>::MINB) fwd_kernel(const FwdParams p) {
  using E = Elt<BF16>;
  constexpr int NW = FwdTile<D>::NW;
  constexpr int BN = FwdTile<D>::BN;
  constexpr int BM = FwdTile<D>::BM;
  constexpr int KS = D / 16;            // QK^T k-steps (16 along d)
  constexpr int NT = BN / 32;           // 32-key subtiles per K/V tile
  constexpr int NP = D / 32;            // 32-wide d panels == PV output tiles
  constexpr int TILE = BN * D * 2;      // bytes of one K or V tile
  constexpr int PIECES = TILE / 1024;   // 1-KiB LDS-DMA pieces per K (or V) tile
  constexpr int PPW = (PIECES + NW - 1) / NW;
  static_assert(TILE % 1024 == 0, "tile must be whole DMA pieces");
  // Staggered halves (8-wave workgroups): waves 4-7 run the PV of each tile one step late, so on
  // every SIMD one wave opens its step with the softmax VALU while its partner opens with PV MFMAs
  // (MI355X_MICROARCH.md "Two waves per SIMD", item 9).  The late PV reads V(nb-1) while the DMA of
  // V(nb+3) is in flight, hence a 5-deep V ring next to the 4-deep K ring.
  // (Round 4, when dropout still staged its random bytes in LDS: unstaggered with a 4-deep V ring
  // measured 7 % slower at d = 64 with dropout, tools/ab.py 2.205 vs 2.060 ms: kept staggered.)
  constexpr bool STAGGER = NW == 8;
  constexpr int VBUFS = STAGGER ? 5 : 4;
  constexpr int VBASE = kFwdBufs * TILE;
  constexpr int SCRATCH = VBASE + VBUFS * TILE;
  constexpr int LDS_BYTES = SCRATCH;   // [K ring][V ring]
  __shared__ __attribute__((aligned(16))) char smem[LDS_BYTES];
  auto kslot = [&](int nb) { return (nb % kFwdBufs) * TILE; };
  auto vslot = [&](int nb) { return VBASE + (nb % VBUFS) * TILE; };

  const AttnShape s = p.s;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = wave_uniform(tid >> 6);
  const int r = lane & 31, hh = lane >> 5;
  const LdsBases lb(lane);

  // Work order: XCD-aware, heads grouped (xcd_order_grouped, p.head_group from launch_fwd): a few
  // heads' query blocks run together on one XCD, heaviest first, sharing K/V through its L2; the
  // group size bounds the causal tail (all heads of an XCD in sequence, xcd_order, measured -5%).
  int bh, m_idx;
  xcd_order_grouped(blockIdx.x, s.b * s.h, p.num_m_blocks, p.head_group, bh, m_idx);
  const int bidb = bh / s.h;
  const int head = bh - bidb * s.h;
  const int kvh = head / (s.h / s.hk);
  const int m_block = p.num_m_blocks - 1 - m_idx;   // heaviest causal query block of a head first

  // ---- sequence geometry (reference BlockInfo, block_info.h:14-31) ----
  int sq = s.seqlen_q, sk = s.seqlen_k;
  int64_t q_off = (int64_t)bidb * p.q_batch, o_off = (int64_t)bidb * p.o_batch;
  int64_t k_off = (int64_t)bidb * p.k_batch, v_off = (int64_t)bidb * p.v_batch;
  if (s.cu_seqlens_q) {
    const int c0 = s.cu_seqlens_q[bidb];
    sq = s.cu_seqlens_q[bidb + 1] - c0;
    if (!s.varlen_padded_input) { q_off = (int64_t)c0 * p.q_row; o_off = (int64_t)c0 * p.o_row; }
  }
  if (s.cu_seqlens_k) {
    const int c0 = s.cu_seqlens_k[bidb];
    sk = s.cu_seqlens_k[bidb + 1] - c0;
    if (!s.varlen_padded_input) { k_off = (int64_t)c0 * p.k_row; v_off = (int64_t)c0 * p.v_row; }
  }
  if (p.rng_state != nullptr && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) {
    p.rng_state[0] = p.seed;
    p.rng_state[1] = p.offset;
  }
  const int m0 = m_block * BM;
  if (m0 >= sq) return;
  if constexpr (SPLIT) {   // this workgroup's key range
    static_assert(!CAUSAL && !DROPOUT && !MASKED, "split-KV is for plain non-causal launches");
    const int n0s = blockIdx.y * p.split_tiles * BN;
    k_off += (int64_t)n0s * p.k_row;
    v_off += (int64_t)n0s * p.v_row;
    sk = max(0, min(sk - n0s, p.split_tiles * BN));
  }

  typedef unsigned short u16;
  const int G = SPLIT ? p.pack_g : 1;   // packed query heads per row group (split-KV path)
  const u16* __restrict__ Q = (const u16*)p.q + q_off + (int64_t)head * G * p.q_head;
  const u16* __restrict__ K = (const u16*)p.k + k_off + (int64_t)kvh * p.k_head;
  const u16* __restrict__ V = (const u16*)p.v + v_off + (int64_t)kvh * p.v_head;
  u16* __restrict__ O = (u16*)p.o + o_off + (int64_t)head * p.o_head;
  float* __restrict__ LSE = p.lse + ((int64_t)bidb * s.h + head) * s.lse_pitch;

  const int wq0 = m0 + 32 * wave;   // first query row of this wave
  const int qi = wq0 + r;           // this lane's query row
  const int dlim = s.d;

  // ---- Q fragments (B operand of S^T = K Q^T): lane holds Q[qi][16ks + 8hh .. +7] ----
  i16x8_t qf[KS];
  {
    const bool ok = qi < sq;
    const u16* qrow = SPLIT ? Q + (int64_t)(ok ? qi / G : 0) * p.q_row + (int64_t)(ok ? qi % G : 0) * p.q_head
                            : Q + (int64_t)(ok ? qi : 0) * p.q_row;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int d0 = 16 * ks + 8 * hh;
      qf[ks] = __builtin_bit_cast(i16x8_t, ld16(qrow + d0, ok && d0 < dlim));
    }
  }

  const int n_end = CAUSAL ? min(sk, m0 + BM) : sk;
  const int nblk = n_end > 0 ? (n_end + BN - 1) / BN : 0;
  // tiles [0, nfast) need no mask for any row of the workgroup (none at all with a dense mask or
  // FlashMask)
  const int nfast = MASKED ? 0 : min(nblk, (CAUSAL ? min(sk, m0 + 1) : sk) / BN);

  // ---- LDS-DMA of K/V tiles: per-lane byte offsets of this wave's 1-KiB pieces ----
  // piece pc covers rows 16*(pc % (BN/16)) .. +15 of panel pc / (BN/16); lane l writes
  // (row = l/4, slot = l%4), i.e. logical chunk slot ^ ((row >> 2) & 3) (panel XOR swizzle).
  int voff_k[PPW], voff_v[PPW];
#pragma unroll
  for (int j = 0; j < PPW; ++j) {
    const int pc = wave + j * NW;
    const int panel = pc / (BN / 16);
    const int row = (pc % (BN / 16)) * 16 + (lane >> 2);
    const int col = panel * 32 + (((lane & 3) ^ ((row >> 2) & 3)) << 3);
    const bool ok = col < dlim;
    voff_k[j] = ok ? (int)(((int64_t)row * p.k_row + col) * 2) : 0x7ffffff0;
    voff_v[j] = ok ? (int)(((int64_t)row * p.v_row + col) * 2) : 0x7ffffff0;
  }
  // DMA of K/V tile `nb` into ring position `pos` (the same except when FlashMask skips tiles)
  auto issue_at = [&](int nb, int pos) {
    const int n0 = nb * BN;
    char* kdst = smem + kslot(pos);
    char* vdst = smem + vslot(pos);
    const int64_t kb = (int64_t)(sk - n0) * p.k_row * 2, vb = (int64_t)(sk - n0) * p.v_row * 2;
    const int krec = (int)(kb > 0x7fffffff ? 0x7fffffff : kb);
    const int vrec = (int)(vb > 0x7fffffff ? 0x7fffffff : vb);
    const buf_rsrc_t rk = make_rsrc(K + (int64_t)n0 * p.k_row, krec);
    const buf_rsrc_t rv = make_rsrc(V + (int64_t)n0 * p.v_row, vrec);
#pragma unroll
    for (int j = 0; j < PPW; ++j) {
      const int pc = wave + j * NW;
      if (PIECES % NW == 0 || pc < PIECES) {
        dma16(rk, kdst + pc * 1024, voff_k[j]);
        dma16(rv, vdst + pc * 1024, voff_v[j]);
      }
    }
  };
  auto issue = [&](int nb) { issue_at(nb, nb); };

  // FlashMask tile skip: a tile is dead when the bounds hide every key of it from every row
  // [m0, min(m0 + BM, sq)) of the workgroup (fm_tile_dead).  Every wave reduces the same bounds, so
  // all waves walk the same sequence of live tiles; dead tiles are neither loaded nor computed.
  const int64_t fmb = (MASKED && s.fm_lts) ? fm_base(s, bidb, head) : 0;
  auto fm_dead = [&](int nb) {
    return fm_tile_dead<CAUSAL>(s, fmb, nb * BN, BN, sk, m0, min(m0 + BM, sq), lane);
  };
  // next live tile after nb (nblk when none)
  auto next_live = [&](int nb) {
    if (nb >= nblk) return nblk;
    ++nb;
    if constexpr (MASKED)
      if (s.fm_lts != nullptr)
        while (nb < nblk && fm_dead(nb)) ++nb;
    return nb;
  };
  // DMA operations one issue() leaves outstanding in this wave.  Step nb reads tiles nb (V) and
  // nb+1 (K, software-pipelined QK^T) and issues nb+3; it ends waiting for nb+2 only, so nb+3
  // stays in flight across the barrier.
  int ndma = 0;
#pragma unroll
  for (int j = 0; j < PPW; ++j)
    if (PIECES % NW == 0 || wave + j * NW < PIECES) ndma += 2;
  auto tile_sync = [&](bool ahead) { wait_dma_keep_and_barrier(ahead ? ndma : 0); };

  // S^T = K Q^T for the tile in buffer kt (K fragments issued in groups of KG ahead of their MFMAs)
  constexpr int KG = (KS % 4 == 0) ? 4 : ((KS % 3 == 0) ? 3 : 2);
  static_assert(KS % KG == 0, "K fragment group must divide the k-steps");
  auto qk = [&](int kt_off, f32x16_t (&st)[NT]) {
    const TileAddr ta(lb, kt_off);
    static_for<0, NT>([&](auto T) {
      constexpr int t = decltype(T)::value;
#pragma unroll
      for (int g = 0; g < 16; ++g) st[t][g] = 0.f;
      static_for<0, KS / KG>([&](auto GG) {
        constexpr int g0 = decltype(GG)::value * KG;
        i16x8_t ka[KG];
        static_for<0, KG>([&](auto KK) {
          constexpr int ks = g0 + decltype(KK)::value;
          ka[ks - g0] = row_read_c<BN, t * 32, 2 * ks>(smem, ta);
        });
#pragma unroll
        for (int k = 0; k < KG; ++k) st[t] = E::mfma(ka[k], qf[g0 + k], st[t]);
      });
    });
  };
  auto rowmax = [&](const f32x16_t (&st)[NT]) {
    float mx[4] = {kNegInf, kNegInf, kNegInf, kNegInf};
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int g = 0; g < 16; ++g) mx[g & 3] = fmaxf(mx[g & 3], st[t][g]);
    return half_swap_max(fmaxf(fmaxf(mx[0], mx[1]), fmaxf(mx[2], mx[3])));
  };

  float m_run = kNegInf, l_run = 0.f;
  f32x16_t o[NP];
#pragma unroll
  for (int t = 0; t < NP; ++t)
#pragma unroll
    for (int g = 0; g < 16; ++g) o[t][g] = 0.f;
  const float c = s.scale_log2;

  // online-softmax update for a tile whose row max (incl. the other lane half) is mt
  auto rescale = [&](float mt) {
    const float m_new = fmaxf(m_run, mt);
    // deferred max (T13): keep the running max while no row of the wave grew by more than
    // kFwdRescaleThr (log2 units), so P <= 2^kFwdRescaleThr; the first finite tile always rescales
    if (__any(m_run == kNegInf ? m_new != m_run : (mt - m_run) * c > kFwdRescaleThr)) {
      const float alpha = fast_exp2(m_run * c - ((m_new == kNegInf) ? 0.f : m_new * c));
      l_run *= alpha;
#pragma unroll
      for (int t = 0; t < NP; ++t)
#pragma unroll
        for (int g = 0; g < 16; ++g) o[t][g] *= alpha;
      m_run = m_new;
    }
  };
  // P = exp2(S c - m c) -> packed B operands; adds the partial row sum of this lane to l_run (the
  // sum is over the undropped P, as in the reference); with dropout the dropped elements of the
  // packed P are zero (reference flash_fwd_kernel.h:429-432; O is scaled by 1/keep_prob at the end)
  const uint64_t doff = s.philox_offset + (uint64_t)(bidb * s.h + head) * 32;
  // dropout bytes of the tile at key n0, in registers (dropout_lane_bytes: one Philox call per lane
  // and 32-key subtile, the bytes of the lane's own scores swapped in from lane ^ 8 by DPP; no LDS
  // scratch and no LDS drain per tile); the refit path reuses them
  typedef unsigned DropBytes[NT][4];
  auto gen_bytes = [&](DropBytes& db, int n0) {
    if constexpr (DROPOUT) {
#pragma unroll
      for (int t = 0; t < NT; ++t) dropout_lane_bytes(db[t], s.philox_seed, doff, wq0, n0 + 32 * t, lane);
    }
    (void)db; (void)n0;
  };
  auto softmax_pack = [&](f32x16_t (&st)[NT], i16x8_t (&pf)[2 * NT], const DropBytes& db) {
    const float ms = (m_run == kNegInf) ? 0.f : m_run * c;
    float ls[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const unsigned* rb = db[t];
#pragma unroll
      for (int g = 0; g < 16; ++g) {
        const float pv = fast_exp2(fmaf(st[t][g], c, -ms));
        ls[g & 3] += pv;
        if constexpr (DROPOUT) st[t][g] = dropout_keep(rb[g >> 2], g & 3, s.keep_u8) ? pv : 0.f;
        else st[t][g] = pv;
      }
      pf[2 * t] = pack_frag<BF16>(st[t], 0);
      pf[2 * t + 1] = pack_frag<BF16>(st[t], 1);
    }
    l_run += (ls[0] + ls[1]) + (ls[2] + ls[3]);
  };
  // Fast-path softmax, no max pass: P = exp2(S c - m_run c) against the running max of earlier
  // tiles (finite here).  Returns this lane's partial row sum; the caller adds it to l_run only after
  // the overflow check (guard_ok), so a tile that trips the check is simply recomputed.
  auto softmax_fast = [&](const f32x16_t (&st)[NT], i16x8_t (&pf)[2 * NT], const DropBytes& db) {
    const float ms = m_run * c;
    float ls[4];
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const unsigned* rb = db[t];
      f32x16_t pt;
#pragma unroll
      for (int g = 0; g < 16; ++g) {
        pt[g] = fast_exp2(fmaf(st[t][g], c, -ms));
        ls[g & 3] = (t == 0 && g < 4) ? pt[g] : ls[g & 3] + pt[g];
        if constexpr (DROPOUT) pt[g] = dropout_keep(rb[g >> 2], g & 3, s.keep_u8) ? pt[g] : 0.f;
      }
      pf[2 * t] = pack_frag<BF16>(pt, 0);
      pf[2 * t + 1] = pack_frag<BF16>(pt, 1);
    }
    return (ls[0] + ls[1]) + (ls[2] + ls[3]);
  };
  // Deferred max without computing it: while every lane's partial sum of P over the tile stays
  // <= 2^kFwdRescaleThr, every P is <= 2^kFwdRescaleThr (and finite), which is all the deferred-max
  // rule needs.  A tile that exceeds it (a score jump, or +inf) takes the slow path below.
  auto guard_ok = [&](float ls) { return !__any(!(ls <= kFwdSumThr)); };
  // Slow path (wave-uniform, rare): recompute S of tile nb (still resident in the K ring), move the
  // running max to the true max, rescale O / l_run, and redo P.  NaN sums (NaN inputs) also land
  // here and end as the reference's NaN / +inf LSE through the normal epilogue.
  auto refit = [&](int nb, i16x8_t (&pf)[2 * NT], const DropBytes& db) {
    asm volatile("; refit" ::: "memory");   // not speculated into the fast path (if-conversion)
    f32x16_t st[NT];
    qk(kslot(nb), st);
    float mx[4] = {kNegInf, kNegInf, kNegInf, kNegInf};
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int g = 0; g < 16; ++g) mx[g & 3] = fmaxf(mx[g & 3], st[t][g]);
    const float mt = half_swap_max(fmaxf(fmaxf(mx[0], mx[1]), fmaxf(mx[2], mx[3])));
    const float m_new = fmaxf(m_run, mt);
    const float alpha = fast_exp2((m_run - m_new) * c);
    l_run *= alpha;
#pragma unroll
    for (int t = 0; t < NP; ++t)
#pragma unroll
      for (int g = 0; g < 16; ++g) o[t][g] *= alpha;
    m_run = m_new;
    return softmax_fast(st, pf, db);
  };
  // O^T[d][q] += V^T[d][key] P^T[key][q], one 32-wide d tile at a time
  auto pv = [&](int vt_off, const i16x8_t (&pf)[2 * NT]) {
    const TileAddr ta(lb, vt_off);
    static_for<0, NP>([&](auto DTC) {
      constexpr int dt = decltype(DTC)::value;
      i16x8_t a[2 * NT];
      static_for<0, 2 * NT>([&](auto KC) {
        constexpr int kk = decltype(KC)::value;
        a[kk] = tr_frag_c<BN, kk * 16, dt>(smem, ta);
      });
#pragma unroll
      for (int kk = 0; kk < 2 * NT; ++kk) o[dt] = E::mfma(a[kk], pf[kk], o[dt]);
    });
  };

  if (wave >= NW / 2) __builtin_amdgcn_s_setprio(1);   // younger half: static priority (T5 static form)
  // tiles at ring positions 0, 1, 2 (0, 1, 2 unless FlashMask skips tiles)
  const int tq0 = next_live(-1), tq1 = next_live(tq0), tq2 = next_live(tq1);
  if (tq0 < nblk) issue_at(tq0, 0);
  if (tq1 < nblk) issue_at(tq1, 1);
  wait_vmem_all();   // Q fragments, tiles 0 and 1 (compiler-visible: no vmcnt waits inside the loops)
  if (tq2 < nblk) issue_at(tq2, 2);
  lds_barrier();

  // ---- fast path: unmasked tiles, QK^T of the next tile overlapped with this tile's softmax ----
  if (!MASKED && nfast > 0) {
    f32x16_t sa[NT], sb[NT];
    qk(kslot(0), sa);
    rescale(rowmax(sa));   // first tile: running max from an explicit max pass
    auto body = [&](int nb, f32x16_t (&scur)[NT], f32x16_t (&snxt)[NT]) {
      if (nb + 3 < nblk) issue(nb + 3);
      i16x8_t pf[2 * NT];
      DropBytes db;
      gen_bytes(db, nb * BN);
      float ls = softmax_fast(scur, pf, db);
      // tile nb+1 is resident (possibly past nblk: then its scores are simply discarded); its
      // MFMAs are independent of the softmax above, so the two interleave in this basic block
      qk(kslot(nb + 1), snxt);
      if (!guard_ok(ls)) ls = refit(nb, pf, db);
      l_run += ls;
      __builtin_amdgcn_sched_barrier(0);   // bound the V-read hoisting (register pressure)
      pv(vslot(nb), pf);
      tile_sync(nb + 3 < nblk);
    };
    // staggered half: PV(nb-1) first (its P fragments carried across the barrier), then the
    // softmax of nb and QK(nb+1); a refit of nb follows the late PV, so O is complete up to nb-1
    // whenever it is scaled
    i16x8_t pfp[2 * NT];
    auto body_late = [&](int nb, f32x16_t (&scur)[NT], f32x16_t (&snxt)[NT]) {
      if (nb + 3 < nblk) issue(nb + 3);
      if (nb > 0) pv(vslot(nb - 1), pfp);
      __builtin_amdgcn_sched_barrier(0);
      DropBytes db;
      gen_bytes(db, nb * BN);
      float ls = softmax_fast(scur, pfp, db);
      qk(kslot(nb + 1), snxt);
      if (!guard_ok(ls)) ls = refit(nb, pfp, db);
      l_run += ls;
      tile_sync(nb + 3 < nblk);
    };
    int nb = 0;
    if (!STAGGER || wave < NW / 2) {
      for (; nb + 1 < nfast; nb += 2) {
        body(nb, sa, sb);
        body(nb + 1, sb, sa);
      }
      if (nb < nfast) body(nb, sa, sb);
    } else {
      for (; nb + 1 < nfast; nb += 2) {
        body_late(nb, sa, sb);
        body_late(nb + 1, sb, sa);
      }
      if (nb < nfast) body_late(nb, sa, sb);
      pv(vslot(nfast - 1), pfp);   // the last deferred PV (V(nfast-1) is not overwritten before
                                   // the general path's issue(nfast+3) lands in another slot)
    }
  }

  // ---- general path: causal diagonal / ragged tiles, per-element masks ----
  // ring position pos holds tile nb; a1, a2 are the next two live tiles (already in flight)
  int nb = MASKED ? tq0 : nfast, a1 = MASKED ? tq1 : nfast + 1, a2 = MASKED ? tq2 : nfast + 2;
  for (int pos = nfast; nb < nblk; ++pos) {
    const int n0 = nb * BN;
    const int a3 = next_live(a2);
    if (a3 < nblk) issue_at(a3, pos + 3);
    const bool active = (wq0 < sq) && (!CAUSAL || n0 <= wq0 + 31);
    if (active) {
      DropBytes db;
      gen_bytes(db, n0);
      f32x16_t st[NT];
      qk(kslot(pos), st);
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int g = 0; g < 16; ++g) {
          const int key = n0 + t * 32 + acc_row(g, hh);
          if (key >= sk || (CAUSAL && key > qi)) st[t][g] = kNegInf;
        }
      if constexpr (MASKED) {
        const u16* mrow = mask_row_ptr(s, bidb, head, qi < sq ? qi : 0);
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
          for (int g = 0; g < 16; ++g) {
            const int key = n0 + t * 32 + acc_row(g, hh);
            if (key >= sk || (CAUSAL && key > qi)) continue;
            if (s.fm_lts != nullptr && fm_masked<CAUSAL>(s, fmb + key, qi)) st[t][g] = kNegInf;
            else if (mrow != nullptr) st[t][g] += E::to_f32(mrow[key]) * s.mask_unscale;
          }
      }
      rescale(rowmax(st));
      i16x8_t pf[2 * NT];
      softmax_pack(st, pf, db);
      pv(vslot(pos), pf);
    }
    tile_sync(a3 < nblk);
    nb = a1; a1 = a2; a2 = a3;
  }

  // ---- epilogue ----
  const float l_tot = half_swap_sum(l_run);
  const bool bad = (l_tot == 0.f) || (l_tot != l_tot);
  const float inv = bad ? 1.f : fast_rcp(l_tot) * (DROPOUT ? s.rp_dropout : 1.f);
  const float lse = bad ? __builtin_huge_valf() : m_run * s.scale + __logf(l_tot);
  if constexpr (SPLIT) {
    // fp32 partial O_i = O / l and LSE_i (-inf for an empty range, NaN propagates) for the combine
    if (qi < sq) {
      const int64_t prow = ((int64_t)blockIdx.y * s.b * s.h + bh) * s.seqlen_q + qi;
      float* arow = p.o_acc + prow * p.acc_d;
      const float iv = l_tot == 0.f ? 0.f : fast_rcp(l_tot);
#pragma unroll
      for (int dt = 0; dt < NP; ++dt)
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int col = dt * 32 + 8 * u + 4 * hh;
          if (col < dlim) {
            const f32x4_t w = {o[dt][4 * u] * iv, o[dt][4 * u + 1] * iv, o[dt][4 * u + 2] * iv,
                               o[dt][4 * u + 3] * iv};
            *(f32x4_t*)(arow + col) = w;
          }
        }
      if (hh == 0) p.lse_acc[prow] = l_tot == 0.f ? -__builtin_huge_valf() : m_run * s.scale + __logf(l_tot);
    }
    return;
  }
  {
    // 16-byte stores: v_permlane32_swap pairs column groups (u, u+1) so that lane half 0 holds
    // columns 8u..8u+7 and half 1 columns 8u+8..8u+15 of its row (T21)
    u16* orow = O + (int64_t)(qi < sq ? qi : 0) * p.o_row;
#pragma unroll
    for (int dt = 0; dt < NP; ++dt)
#pragma unroll
      for (int u = 0; u < 4; u += 2) {
        unsigned a0 = E::pack2(o[dt][4 * u + 0] * inv, o[dt][4 * u + 1] * inv);
        unsigned a1 = E::pack2(o[dt][4 * u + 2] * inv, o[dt][4 * u + 3] * inv);
        unsigned b0 = E::pack2(o[dt][4 * u + 4] * inv, o[dt][4 * u + 5] * inv);
        unsigned b1 = E::pack2(o[dt][4 * u + 6] * inv, o[dt][4 * u + 7] * inv);
        auto r0 = __builtin_amdgcn_permlane32_swap(a0, b0, false, false);
        auto r1 = __builtin_amdgcn_permlane32_swap(a1, b1, false, false);
        const int col = dt * 32 + 8 * u + 8 * hh;
        if (qi < sq && col < dlim) {
          u32x4_t w = {(unsigned)r0[0], (unsigned)r1[0], (unsigned)r0[1], (unsigned)r1[1]};
          *(u32x4_t*)(orow + col) = w;
        }
      }
    if (qi < sq && hh == 0) LSE[qi] = lse;
  }
}

// return_softmax (test-only, reference flash_api.cpp:276-279): S_dmask[b][h][i][j] =
// exp(scale * (q_i . k_j + mask_ij * unscale) - LSE_i), negated where dropout drops the element, 0
// where causal / FlashMask hides it or it is padding (the reference writes P in its dense-mask and
// FlashMask kernels too, flash_fwd_kernel.h:880-887, 1513-1520).  A plain fp32 dot product per
// element: it runs only for the reference's dropout tests.
template <bool BF16>
__global__ void __launch_bounds__(256) dmask_kernel(const FwdParams p) {
  using E = Elt<BF16>;
  typedef unsigned short u16;
  const AttnShape s = p.s;
  const int bh = blockIdx.z;
  const int bidb = bh / s.h, head = bh - bidb * s.h;
  const int kvh = head / (s.h / s.hk);
  const int col = blockIdx.x * 64 + (threadIdx.x & 63);
  const int row = blockIdx.y * 4 + (threadIdx.x >> 6);
  if (row >= p.p_rows || col >= p.p_cols) return;
  int sq = s.seqlen_q, sk = s.seqlen_k;
  int64_t q_off = (int64_t)bidb * p.q_batch, k_off = (int64_t)bidb * p.k_batch;
  if (s.cu_seqlens_q) {
    const int c0 = s.cu_seqlens_q[bidb];
    sq = s.cu_seqlens_q[bidb + 1] - c0;
    if (!s.varlen_padded_input) q_off = (int64_t)c0 * p.q_row;
  }
  if (s.cu_seqlens_k) {
    const int c0 = s.cu_seqlens_k[bidb];
    sk = s.cu_seqlens_k[bidb + 1] - c0;
    if (!s.varlen_padded_input) k_off = (int64_t)c0 * p.k_row;
  }
  float val = 0.f;
  bool live = row < sq && col < sk && !(s.causal && col > row);
  if (live && s.fm_lts != nullptr) {
    const int64_t c = fm_base(s, bidb, head) + col;
    live = !(s.causal ? fm_masked<true>(s, c, row) : fm_masked<false>(s, c, row));
  }
  if (live) {
    const u16* qr = (const u16*)p.q + q_off + (int64_t)head * p.q_head + (int64_t)row * p.q_row;
    const u16* kr = (const u16*)p.k + k_off + (int64_t)kvh * p.k_head + (int64_t)col * p.k_row;
    float acc = 0.f;
    for (int d = 0; d < s.d; ++d) acc += E::to_f32(qr[d]) * E::to_f32(kr[d]);
    const u16* mrow = mask_row_ptr(s, bidb, head, row);
    if (mrow != nullptr) acc += E::to_f32(mrow[col]) * s.mask_unscale;
    const float lse = p.lse[((int64_t)bidb * s.h + head) * s.lse_pitch + row];
    val = __expf(acc * s.scale - lse);
    // the reference's byte for (row, col), computed directly (one Philox call per element)
    const int rr = row % 16, cc = col % 32;
    const int lanec = 4 * (rr % 8) + (cc % 8) / 2;
    const int bidx = 8 * (cc / 16) + (cc % 2) + 2 * (rr / 8) + 4 * ((cc % 16) / 8);
    const uint64_t sub = (uint64_t)(unsigned)(row / 16) | ((uint64_t)(unsigned)(col / 32) << 32);
    const u32x4_t w = philox(s.philox_seed, sub, s.philox_offset + (uint64_t)bh * 32 + lanec);
    const unsigned byte = (w[bidx >> 2] >> (8 * (bidx & 3))) & 0xffu;
    if (byte > s.keep_u8) val = -val;
  }
  u16* out = (u16*)p.p_out + ((int64_t)bh * p.p_rows + row) * p.p_cols + col;
  *out = (u16)(E::pack2(val, 0.f) & 0xffff);
}

// Split-KV combine: one wave per (b, h, query row).  LSE = log sum_i exp(LSE_i), O = sum_i
// exp(LSE_i - LSE) O_i (the reference's combine_attn_seqk_parallel in FA2's split-KV path, done
// here without its shared-memory transpose: split i's weight is broadcast from lane i).
template <bool BF16>
__global__ void __launch_bounds__(256) splitkv_combine_kernel(const FwdParams p) {
  using E = Elt<BF16>;
  typedef unsigned short u16;
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);   // (b * h) * seqlen_q + q
  const int64_t nrows = (int64_t)p.s.b * p.s.h * p.s.seqlen_q;
  if (row >= nrows) return;
  const int qi = (int)(row % p.s.seqlen_q);   // packed row (query qi / G, head qi % G of the group)
  const int bh = (int)(row / p.s.seqlen_q);
  const int G = p.pack_g;
  const int bidb = bh / p.s.h, kvh = bh - bidb * p.s.h;
  const int q = qi / G, head = kvh * G + qi % G;
  const int64_t split_stride = nrows;
  float li = lane < p.n_split ? p.lse_acc[lane * split_stride + row] : -__builtin_huge_valf();
  float mx = li;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) mx = fmaxf(mx, __shfl_xor(mx, off));
  const bool empty = mx == -__builtin_huge_valf();
  float w = empty ? 0.f : __expf(li - mx);
  float sum = w;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) sum += __shfl_xor(sum, off);
  const float lse = empty ? __builtin_huge_valf() : mx + __logf(sum);
  w = empty ? 0.f : w / sum;
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  for (int i = 0; i < p.n_split; ++i) {
    const float wi = __shfl(w, i);
    const float* src = p.o_acc + (i * split_stride + row) * p.acc_d;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int col = lane + 64 * c;
      if (col < p.s.d && wi != 0.f) acc[c] += wi * src[col];
    }
  }
  u16* orow = (u16*)p.o + (int64_t)bidb * p.o_batch + (int64_t)head * p.o_head + (int64_t)q * p.o_row;
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const int col = lane + 64 * c;
    if (col < p.s.d) orow[col] = (u16)(E::pack2(acc[c], 0.f) & 0xffffu);
  }
  if (lane == 0) p.lse[((int64_t)bidb * p.s.h * G + head) * p.s.lse_pitch + q] = lse;
}

template <bool BF16, int D, bool CAUSAL, bool DROPOUT>
static void run_fwd(const FwdParams& p, hipStream_t stream) {
  dim3 grid(p.s.b * p.s.h * p.num_m_blocks);   // 1-D: heads fastest, heaviest query block first
  prof_begin(kTimeFwd, stream);
  if constexpr (!DROPOUT && (D == 128 || D == 64)) {   // hand-scheduled assembly kernels (fa_fwd_asm.cpp)
    // the persistent assembly forward groups heads per XCD below the Infinity-Cache threshold too
    // (knob 7): a head's K/V is then streamed by many CUs of one XCD at once and served from its L2
    // (C3: forward -0.5 to -0.9 %, profiles/r04/ab_asm_xcd_group_c3_r04e.txt)
    FwdParams pa = p;
    if (pa.n_split == 0 && pa.pack_g == 1 && p.s.cu_seqlens_q == nullptr)   // (varlen: device-built list)
      pa.head_group = xcd_head_group((long long)p.s.b * p.s.h, p.num_m_blocks, 4ll * p.s.b * p.s.seqlen_k * p.s.hk * p.s.d,
                                     p.s.causal, knob(kKnobAsmXcdGroupMinMiB));
    if (launch_fwd_asm(pa, BF16, stream)) {
      prof_end(kTimeFwd, stream);
      return;
    }
  }
  if constexpr (!CAUSAL && !DROPOUT) {
    if (p.n_split > 0) {
      hipLaunchKernelGGL((fwd_kernel<BF16, D, false, false, false, true>), dim3(grid.x, p.n_split),
                         dim3(FwdTile<D>::NW * 64), 0, stream, p);
      const int64_t rows = (int64_t)p.s.b * p.s.h * p.s.seqlen_q;
      hipLaunchKernelGGL((splitkv_combine_kernel<BF16>), dim3((unsigned)((rows + 3) / 4)), dim3(256), 0,
                         stream, p);
      prof_end(kTimeFwd, stream);
      return;
    }
  }
  if (p.s.mask != nullptr || p.s.fm_lts != nullptr)
    hipLaunchKernelGGL((fwd_kernel<BF16, D, CAUSAL, DROPOUT, true>), grid, dim3(FwdTile<D>::NW * 64), 0, stream, p);
  else
    hipLaunchKernelGGL((fwd_kernel<BF16, D, CAUSAL, DROPOUT, false>), grid, dim3(FwdTile<D>::NW * 64), 0, stream, p);
  prof_end(kTimeFwd, stream);
}

template <bool BF16, bool CAUSAL, bool DROPOUT>
static void dispatch_d(const FwdParams& p, hipStream_t stream) {
  const int d = p.s.d;
  if (d <= 32) run_fwd<BF16, 32, CAUSAL, DROPOUT>(p, stream);
  else if (d <= 64) run_fwd<BF16, 64, CAUSAL, DROPOUT>(p, stream);
  else if (d <= 96) run_fwd<BF16, 96, CAUSAL, DROPOUT>(p, stream);
  else if (d <= 128) run_fwd<BF16, 128, CAUSAL, DROPOUT>(p, stream);
  // dedicated tiles (reference hdim160); at 2 x 4096 x 16 causal a d = 160 forward takes the same
  // time on these as on the D = 192 tiles (0.331 / 0.326 ms, tools/hdim_bench.py): not MFMA-bound
  else if (d <= 160) run_fwd<BF16, 160, CAUSAL, DROPOUT>(p, stream);
  else if (d <= 192) run_fwd<BF16, 192, CAUSAL, DROPOUT>(p, stream);
  else if (d <= 224) run_fwd<BF16, 224, CAUSAL, DROPOUT>(p, stream);   // (reference hdim224)
  else if (d <= 256) run_fwd<BF16, 256, CAUSAL, DROPOUT>(p, stream);
  else throw std::runtime_error("flash_attn_fwd: head dim " + std::to_string(d) + " > 256");
}

template <bool BF16>
static void dispatch_fwd(const FwdParams& p, hipStream_t stream) {
  if (p.s.causal) {
    if (p.s.dropout) dispatch_d<BF16, true, true>(p, stream); else dispatch_d<BF16, true, false>(p, stream);
  } else {
    if (p.s.dropout) dispatch_d<BF16, false, true>(p, stream); else dispatch_d<BF16, false, false>(p, stream);
  }
  if (p.p_out != nullptr) {
    dim3 grid((p.p_cols + 63) / 64, (p.p_rows + 3) / 4, p.s.b * p.s.h);
    hipLaunchKernelGGL((dmask_kernel<BF16>), grid, dim3(256), 0, stream, p);
  }
}

void fwd_block_size(int d, int* block_m, int* block_n) {
  *block_m = d <= 64 ? FwdTile<64>::BM : (d <= 128 ? FwdTile<128>::BM : FwdTile<256>::BM);
  *block_n = d <= 64 ? FwdTile<64>::BN : (d <= 128 ? FwdTile<128>::BN : FwdTile<256>::BN);
}

// Split-KV for decode-shaped calls (FA2's num_splits heuristic, flash_api.cpp): with fewer
// workgroups than CUs, split the keys so that about two workgroups per CU stream K/V, each split
// at least 4 tiles; plain non-causal fixed-length launches only.  FLASH_ATTN_MI355X_NO_SPLITKV=1
// disables it (tests compare both paths).
// GQA packing on top (decode with grouped heads): the query heads of a kv head are packed as
// extra rows when seqlen_q * group fits one query block, so K/V are streamed once per kv head.
// Sets n_split / split_tiles / pack_g (and the packed shape); allocates nothing.
static void plan_split(FwdParams& p) {
  p.n_split = 0;   // 0: the ordinary launch
  p.pack_g = 1;
  int bm, bn;
  fwd_block_size(p.s.d, &bm, &bn);
  const int nblk = (p.s.seqlen_k + bn - 1) / bn;
  const bool plain = !p.s.causal && !p.s.dropout && p.s.mask == nullptr && p.s.fm_lts == nullptr &&
                     p.p_out == nullptr && p.s.cu_seqlens_q == nullptr && p.s.cu_seqlens_k == nullptr;
  const int G = p.s.h / p.s.hk;
  const bool pack = plain && G > 1 && (long long)p.s.seqlen_q * G <= bm;
  const long long wgs = pack ? (long long)p.s.b * p.s.hk : (long long)p.s.b * p.s.h * p.num_m_blocks;
  if (plain && knob(kKnobNoSplitKv) != 1 && nblk > 0 && (pack || (wgs < 256 && nblk >= 8))) {
    int ns = 1;
    if (wgs < 256 && nblk >= 8)
      ns = (int)std::min<long long>(64, std::min<long long>((512 + wgs - 1) / wgs, nblk / 4));
    if (ns >= 2 || pack) {
      p.split_tiles = (nblk + ns - 1) / ns;
      p.n_split = (nblk + p.split_tiles - 1) / p.split_tiles;
      if (pack) {
        p.pack_g = G;
        p.s.h = p.s.hk;
        p.s.seqlen_q *= G;
        p.num_m_blocks = 1;
      }
      p.head_group = 0;
    }
  }
}

// (fa_params.h: a pure function of the call.)  Head dim 64 / 128 without dropout -- the assembly
// forward's domain, plus the dense mask and FlashMask, whose calls run the HIP kernels on Q' so that
// a mask that hides nothing gives the unmasked call's result (the mask term enters the log2-domain
// scores as mask * unscale * c); fp16 only with |c| <= 1, where c Q cannot overflow the 16-bit Q'.
// Dropout calls (HIP kernels only) keep the exact Q: a fold would cost them a Q' pass for nothing.
// FLASH_ATTN_MI355X_NO_QFOLD=1 (read once per process, so a forward and its backward always agree)
// scores every call from the exact Q: the reference's precision class, at +5 % forward / +2 % dK/dV
// time at C3 (profiles/r06/ab_c3_nofold_r06n.txt).  The fold's extra rounding of c Q matters only
// where |c q.k| is large and a row has few keys (DESIGN.md deviation 8).
bool attn_folds_q(const AttnShape& s, bool is_bf16) {
#ifdef FA_NO_QFOLD   // (A/B variants whose assembly forward is generated with FA_GEN_FOLD=0)
  return false;
#endif
  static const bool no_fold = [] {
    const char* e = std::getenv("FLASH_ATTN_MI355X_NO_QFOLD");
    return e != nullptr && e[0] == '1';
  }();
  return !no_fold && (s.d == 128 || s.d == 64) && !s.dropout && (is_bf16 || std::fabs(s.scale_log2) <= 1.0f);
}

void launch_fwd(const FwdParams& p_in, bool is_bf16, hipStream_t stream) {
  FwdParams p = p_in;
  if (p.s.b <= 0 || p.s.h <= 0) return;
  p.head_group = xcd_head_group((long long)p.s.b * p.s.h, p.num_m_blocks,
                                 4ll * p.s.b * p.s.seqlen_k * p.s.hk * p.s.d, p.s.causal);   // K + V bytes
#ifdef FA_FWD_NOGROUP
  p.head_group = 0;
#endif
  if (p.num_m_blocks <= 0) return;
  if ((int64_t)p.s.b * p.s.h * p.num_m_blocks > 0x7fffffff)
    throw std::runtime_error("flash_attn_fwd: batch * heads * query blocks too large for the grid");
  StreamScratch ws, qf;
  if (attn_folds_q(p.s, is_bf16)) {
    FwdParams t = p;
    plan_split(t);
    if (!fwd_asm_applicable(t, is_bf16)) {
      // A folding call the assembly kernel does not take (a knob, split-KV, return_softmax, record
      // limits): the HIP kernels score from a materialised Q' with c = 1, scale = ln 2 -- the same
      // scores, LSE and P (S_dmask included) the assembly forward and the backward use.
      const int64_t hd = (int64_t)p.s.h * p.s.d;
      if (!qf.alloc((size_t)p.s.b * p.s.seqlen_q * hd * 2, stream))
        throw std::runtime_error("flash_attn_fwd: hipMallocAsync of the prescaled Q failed");
      QFoldArgs a;
      a.q = p.q; a.qf = qf.p;
      a.q_batch = p.q_batch; a.q_row = p.q_row; a.q_head = p.q_head;
      a.cu_seqlens_q = p.s.cu_seqlens_q; a.padded = p.s.varlen_padded_input;
      a.b = p.s.b; a.seqlen_q = p.s.seqlen_q; a.h = p.s.h; a.d = p.s.d;
      a.c = p.s.scale_log2;
      launch_q_fold(a, is_bf16, stream);
      p.q = qf.p;
      p.q_batch = (int64_t)p.s.seqlen_q * hd; p.q_row = hd; p.q_head = p.s.d;
      p.s.mask_unscale *= p.s.scale_log2;
      p.s.scale = kLn2;
      p.s.scale_log2 = 1.0f;
    }
  }
  plan_split(p);
  if (p.n_split > 0) {
    p.acc_d = (p.s.d + 31) / 32 * 32;
    const size_t rows = (size_t)p.n_split * p.s.b * p.s.h * p.s.seqlen_q;
    const size_t bytes = rows * p.acc_d * sizeof(float) + rows * sizeof(float);
    if (!ws.alloc(bytes, stream))
      throw std::runtime_error("flash_attn_fwd: hipMallocAsync of the split-KV scratch failed");
    p.o_acc = static_cast<float*>(ws.p);
    p.lse_acc = p.o_acc + rows * p.acc_d;
  }
  if (p.p_out != nullptr && (p.p_rows > 65535 * 4 || p.s.b * p.s.h > 65535))
    throw std::runtime_error("flash_attn_fwd: return_softmax grid too large");
  if (is_bf16) dispatch_fwd<true>(p, stream); else dispatch_fwd<false>(p, stream);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string("flash_attn_fwd launch: ") + hipGetErrorString(e));
}

}  // namespace fa
