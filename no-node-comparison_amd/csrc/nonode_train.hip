// EGNO training path on gfx950: forward with saved states + hand-written backward.
//
// Replaces loss.backward() of run_epoch (main_simulation_simple_no.py:267-280) through
// EGNO.forward (egno.py:37-111). The reverse pass follows oracle/egno_grad.py op by op, which is
// pinned to the reference's own autograd gradients (tests/golden/egno_grad.npz).
//
// Included at the end of nonode.hip (same translation unit: shares the ECL helpers, the MFMA
// fragment layout and the launch utilities); node_bwd_kernel is in nonode_node.hip.
//
// Per layer l (reverse order), given the gradients of that layer's outputs (gx, gv, gh):
//   node_bwd_kernel   x/v update + node MLP reverse (basic.py:174-185): gF, gM, gv, part of gh
//   edge_bwd_kernel   per-edge recompute + reverse of the coordinate and edge MLPs (basic.py:
//                     170-173, 107-144): per-receiver / per-sender sums GA, GB and gx terms
//   node_wgrad_kernel gh = part + W_A^T GA + W_B^T GB,  gx = gx + edge terms (and the node-level GEMMs)
//   tconvx_bwd / tconv_bwd  TimeConv_x / TimeConv reverse (layer_no.py:80-178)
// Weight gradients are sums over edges or nodes, C = sum_k G[k] (x) A[k]: the kernels above keep
// per-workgroup partials and gemm_reduce_batch adds them in a fixed order (deterministic).

#include "nonode_bwd_common.h"

namespace {

using nonode_tu::NodeBwdArgs;
using nonode_tu::launch_node_bwd;
using nonode_tu::MMAX_T;
using nonode_tu::TB_MAX_BLOCKS;
using nonode_tu::TconvBwdArgs;
using nonode_tu::launch_tconv_bwd;
using nonode_tu::tb_groups;

// scheduling fence between the pair loop's stages (each stage's two chains interleave, the stages do not)
#define PAIR_FENCE() __builtin_amdgcn_sched_barrier(0)

// frag of W^T: value W^T[row][col] = W[col][row0 + row] (W row stride ld)
__device__ __forceinline__ void pack_frag_t(float* dst, const float* W, int ld, int row0, int d) {
  const int q = d & 3, l = (d >> 2) & 63, rest = d >> 8;
  const int mt = rest & 3, mo = rest >> 2;
  const int row = 16 * mo + (l & 15), col = 16 * mt + 4 * (l >> 4) + q;
  dst[d] = W[col * ld + row0 + row];
}

// pack_h16 of W^T: W^T[row][col] = W[col][row] (W row stride ld; null W: zeros), lo part x 2^k (h8_scale)
__device__ __forceinline__ void pack_h16_t(_Float16* dst, const float* W, int d, int ld, int k) {
  const int j = d & 7, lane = (d >> 3) & 63, hl = (d >> 9) & 1, mo = (d >> 10) & 3, s = d >> 12;
  const int row = 16 * mo + (lane & 15);
  const int col = 16 * (2 * s + (j >> 2)) + 4 * (lane >> 4) + (j & 3);
  const float w = W ? W[col * ld + row] : 0.f;
  const _Float16 h = (_Float16)w;
  dst[d] = hl == 0 ? h : (_Float16)__builtin_ldexpf(w - (float)h, k);   // (see pack_h16)
}
// (of the 64x64 block W[0..63][col0 .. col0+63])
__device__ __forceinline__ void pack_h16_t_shifted(_Float16* dst, float* scal, int idx, const float* W, int d,
                                                   int ld = 64, int col0 = 0) {
  const int k = h16_lo_shift(W, ld, col0, 1.f);   // the transpose has the same largest |element|
  pack_h16_t(dst, W ? W + col0 : W, d, ld, k);
  if (blockIdx.x == 0 && threadIdx.x == 0) scal[SC_H16S + idx] = h16_us_bits(k);
}

__global__ void pack_bwd_kernel(PackBatch pb) {
  const PackArgs& a = pb.a[blockIdx.z];
  const int d = blockIdx.x * blockDim.x + threadIdx.x;   // 0 .. 8191
  float* B = a.blob;
  _Float16* H = reinterpret_cast<_Float16*>(B + BOFF_H16);
  switch (blockIdx.y) {
    case 16: pack_h16_shifted(H + BH_W2 * 8192, B + BOFF_SCAL, BH_W2, a.w2, d); break;
    case 17: pack_h16_shifted(H + BH_WC1 * 8192, B + BOFF_SCAL, BH_WC1, a.cw1, d); break;
    case 18: pack_h16_t_shifted(H + BH_W2T * 8192, B + BOFF_SCAL, BH_W2T, a.w2, d); break;
    case 19: pack_h16_t_shifted(H + BH_WC1T * 8192, B + BOFF_SCAL, BH_WC1T, a.cw1, d); break;
    case 20: pack_h16_shifted(H + BH_WA * 8192, B + BOFF_SCAL, BH_WA, a.w1, d, a.ld1, a.colA); break;
    case 21: pack_h16_shifted(H + BH_WB * 8192, B + BOFF_SCAL, BH_WB, a.w1, d, a.ld1, a.colB); break;
    case 22: pack_h16_shifted(H + BH_WV1 * 8192, B + BOFF_SCAL, BH_WV1, a.vw1, d); break;
    case 23: pack_h16_shifted(H + BH_WN1A * 8192, B + BOFF_SCAL, BH_WN1A, a.nw1, d, 128, 0); break;
    case 24: pack_h16_shifted(H + BH_WN1B * 8192, B + BOFF_SCAL, BH_WN1B, a.nw1, d, 128, HID); break;
    case 25: pack_h16_t_shifted(H + BH_WV1T * 8192, B + BOFF_SCAL, BH_WV1T, a.vw1, d); break;
    case 26: pack_h16_t_shifted(H + BH_WN2T * 8192, B + BOFF_SCAL, BH_WN2T, a.nw2, d); break;
    case 27: pack_h16_t_shifted(H + BH_WN1TH * 8192, B + BOFF_SCAL, BH_WN1TH, a.nw1, d, 128, 0); break;
    case 28: pack_h16_t_shifted(H + BH_WN1TM * 8192, B + BOFF_SCAL, BH_WN1TM, a.nw1, d, 128, HID); break;
    case 29: pack_h16_t_shifted(H + BH_WAT * 8192, B + BOFF_SCAL, BH_WAT, a.w1, d, a.ld1, a.colA); break;
    case 30: pack_h16_t_shifted(H + BH_WBT * 8192, B + BOFF_SCAL, BH_WBT, a.w1, d, a.ld1, a.colB); break;
    case 0: if (d < 4096) pack_frag(B + BOFF_WA, a.w1, a.ld1, a.colA, 4, d, 1.f); break;
    case 1: if (d < 4096) pack_frag(B + BOFF_WB, a.w1, a.ld1, a.colB, 4, d, 1.f); break;
    case 2: if (d < 4096) pack_frag(B + BOFF_W2, a.w2, 64, 0, 4, d, 1.f); break;
    case 3: if (d < 4096) pack_frag(B + BOFF_WC1, a.cw1, 64, 0, 4, d, 1.f); break;
    case 4: if (d < 4096) { if (a.vw1) pack_frag(B + BOFF_WV1, a.vw1, 64, 0, 4, d, 1.f); else B[BOFF_WV1 + d] = 0.f; } break;
    case 5: pack_frag(B + BOFF_WN1, a.nw1, 128, 0, 8, d, 1.f); break;
    case 6: if (d < 4096) pack_frag(B + BOFF_WN2, a.nw2, 64, 0, 4, d, 1.f); break;
    case 7: if (d < 4096) pack_frag_t(B + BOFF_W2T, a.w2, 64, 0, d); break;
    case 8: if (d < 4096) pack_frag_t(B + BOFF_WC1T, a.cw1, 64, 0, d); break;
    case 9: if (d < 4096) { if (a.vw1) pack_frag_t(B + BOFF_WV1T, a.vw1, 64, 0, d); else B[BOFF_WV1T + d] = 0.f; } break;
    case 10: if (d < 4096) pack_frag_t(B + BOFF_WN2T, a.nw2, 64, 0, d); break;
    case 11: if (d < 4096) pack_frag_t(B + BOFF_WN1TH, a.nw1, 128, 0, d); break;
    case 12: if (d < 4096) pack_frag_t(B + BOFF_WN1TM, a.nw1, 128, HID, d); break;
    case 13: if (d < 4096) pack_frag_t(B + BOFF_WAT, a.w1, a.ld1, a.colA, d); break;
    case 14: if (d < 4096) pack_frag_t(B + BOFF_WBT, a.w1, a.ld1, a.colB, d); break;
    case 15:
      if (d < 512) {
        const int kf = d >> 8, l = (d >> 2) & 63, mo = d & 3;
        const int row = 16 * mo + (l & 15), fi = 4 * kf + (l >> 4);
        float val = 0.f;
        if (fi == 0) val = a.w1[row * a.ld1 + a.colS];
        else if (fi - 1 < a.ne) val = a.w1[row * a.ld1 + 2 * HID + 1 + (fi - 1)];
        B[BOFF_FEAT + d] = val;
      } else if (d < 512 + BV_COUNT * 64) {
        const int dd = d - 512, v = dd >> 6, i = dd & 63;
        float val = 0.f;
        switch (v) {
          case BV_B1: val = vp_src(a.b1, 1, i); break;
          case BV_B2: val = vp_src(a.b2, 1, i); break;
          case BV_BC1: val = vp_src(a.cb1, 1, i); break;
          case BV_WC2: val = vp_src(a.cw2, 1, i); break;
          case BV_BV1: val = vp_src(a.vb1, 1, i); break;
          case BV_WV2: val = vp_src(a.vw2, 1, i); break;
          case BV_BN1: val = vp_src(a.nb1, 1, i); break;
          case BV_BN2: val = vp_src(a.nb2, 1, i); break;
          case BV_WS: val = vp_src(a.w1 + a.colS, a.ld1, i); break;
        }
        B[BOFF_VEC + dd] = val;
      } else if (d < 512 + BV_COUNT * 64 + 64) {
        const int i = d - 512 - BV_COUNT * 64;
        float val = 0.f;
        if (i == 0) val = a.cb2[0];
        else if (i == 1 && a.vb2) val = a.vb2[0];
        else if (i == SC_NORM) val = (a.flags & NONODE_LAYER_NORM_RADIAL) ? 1.f : 0.f;
        else if (i == SC_TANH) val = (a.flags & NONODE_LAYER_TANH_COORD) ? 1.f : 0.f;
        if (i < SC_H16S || i >= SC_H16S + BH_COUNT) B[BOFF_SCAL + i] = val;   // shifts: sections 16-30
      }
      break;
  }
}

// out += W x for a gradient column set x: each column scaled to [2^11, 2^12) before the split, the
// product scaled back (per lane: lane (e, g) holds column e)
__device__ __forceinline__ void mm64_cs(f4 (&out)[4], const h8* wh, const f4 (&x)[4], int lane, unsigned us,
                                        float cm) {
  const float sc = p2scale(cm);
  const float inv = 1.f / sc;   // exact (power of two)
  f4 xs[4], acc[4];
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) { xs[mt] = x[mt] * sc; acc[mt] = f4{0.f, 0.f, 0.f, 0.f}; }
  h8 xh[2], xl[2];
  h16_split(xs, xh, xl);
  mfma_h16(acc, wh, xh, xl, lane, us);
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) out[mt] += acc[mt] * inv;
}
__device__ __forceinline__ f4 mfma16k16(h4 a, h4 b, f4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x16f16(a, b, c, 0, 0, 0);
}
// The pair path's weight-gradient MFMAs (wgrad_pair) are inline asm with the accumulators bound to
// AGPRs ("+a"): the library forces VGPR-form MFMAs, which would keep dWc1's 64 accumulator values in
// VGPRs through pass A's pair loop (its register demand then exceeds 512 and LLVM's AGPR-copy rewrite
// crashes). The hazard recognizer does not see inside asm, so each statement carries its own wait
// states: "s_nop 1" first (an accumulator the compiler just wrote or copied, read as C) and "s_nop 11"
// last (12 states: an MFMA result read or copied by compiler code after the statement, the 8-pass XDL
// requirement, more than a 16x16x32 MFMA needs); inside, consecutive MFMAs only chain accumulators.
// One statement = the 12 MFMAs of one output row block (3 fp16x3 terms x 4 column blocks).
__device__ __forceinline__ void amfma32_block(f4 (&acc)[4], h8 al, h8 ah, const h8 (&bh)[4], const h8 (&bl)[4]) {
  asm volatile(
      "s_nop 1\n\t"
      "v_mfma_f32_16x16x32_f16 %0, %4, %6, %0\n\t"
      "v_mfma_f32_16x16x32_f16 %1, %4, %7, %1\n\t"
      "v_mfma_f32_16x16x32_f16 %2, %4, %8, %2\n\t"
      "v_mfma_f32_16x16x32_f16 %3, %4, %9, %3\n\t"
      "v_mfma_f32_16x16x32_f16 %0, %5, %10, %0\n\t"
      "v_mfma_f32_16x16x32_f16 %1, %5, %11, %1\n\t"
      "v_mfma_f32_16x16x32_f16 %2, %5, %12, %2\n\t"
      "v_mfma_f32_16x16x32_f16 %3, %5, %13, %3\n\t"
      "v_mfma_f32_16x16x32_f16 %0, %5, %6, %0\n\t"
      "v_mfma_f32_16x16x32_f16 %1, %5, %7, %1\n\t"
      "v_mfma_f32_16x16x32_f16 %2, %5, %8, %2\n\t"
      "v_mfma_f32_16x16x32_f16 %3, %5, %9, %3\n\t"
      "s_nop 11"
      : "+a"(acc[0]), "+a"(acc[1]), "+a"(acc[2]), "+a"(acc[3])
      : "v"(al), "v"(ah), "v"(bh[0]), "v"(bh[1]), "v"(bh[2]), "v"(bh[3]), "v"(bl[0]), "v"(bl[1]), "v"(bl[2]),
        "v"(bl[3]));
}
// the same for the single-unit form in pass A (K = 16: fp16x3 on v_mfma_f32_16x16x16_f16, operands
// split on the VALU just before: the leading s_nop 1 covers that write)
__device__ __forceinline__ void amfma16_block(f4 (&acc)[4], h4 gl, h4 gh, const h4 (&ah)[4], const h4 (&al)[4]) {
  asm volatile(
      "s_nop 1\n\t"
      "v_mfma_f32_16x16x16_f16 %0, %4, %6, %0\n\t"
      "v_mfma_f32_16x16x16_f16 %1, %4, %7, %1\n\t"
      "v_mfma_f32_16x16x16_f16 %2, %4, %8, %2\n\t"
      "v_mfma_f32_16x16x16_f16 %3, %4, %9, %3\n\t"
      "v_mfma_f32_16x16x16_f16 %0, %5, %10, %0\n\t"
      "v_mfma_f32_16x16x16_f16 %1, %5, %11, %1\n\t"
      "v_mfma_f32_16x16x16_f16 %2, %5, %12, %2\n\t"
      "v_mfma_f32_16x16x16_f16 %3, %5, %13, %3\n\t"
      "v_mfma_f32_16x16x16_f16 %0, %5, %6, %0\n\t"
      "v_mfma_f32_16x16x16_f16 %1, %5, %7, %1\n\t"
      "v_mfma_f32_16x16x16_f16 %2, %5, %8, %2\n\t"
      "v_mfma_f32_16x16x16_f16 %3, %5, %9, %3\n\t"
      "s_nop 11"
      : "+a"(acc[0]), "+a"(acc[1]), "+a"(acc[2]), "+a"(acc[3])
      : "v"(gl), "v"(gh), "v"(ah[0]), "v"(ah[1]), "v"(ah[2]), "v"(ah[3]), "v"(al[0]), "v"(al[1]), "v"(al[2]),
        "v"(al[3]));
}
// exact f32 form (16x16x4 f32), one k-step: acc[ot][it] += gv[ot] av[it]
__device__ __forceinline__ void amfma4_block(f4 (&acc)[4][4], const float (&gv)[4], const float (&av)[4]) {
#pragma unroll
  for (int ot = 0; ot < 4; ++ot)
    asm volatile(
        "s_nop 1\n\t"
        "v_mfma_f32_16x16x4_f32 %0, %4, %5, %0\n\t"
        "v_mfma_f32_16x16x4_f32 %1, %4, %6, %1\n\t"
        "v_mfma_f32_16x16x4_f32 %2, %4, %7, %2\n\t"
        "v_mfma_f32_16x16x4_f32 %3, %4, %8, %3\n\t"
        "s_nop 11"
        : "+a"(acc[ot][0]), "+a"(acc[ot][1]), "+a"(acc[ot][2]), "+a"(acc[ot][3])
        : "v"(gv[ot]), "v"(av[0]), "v"(av[1]), "v"(av[2]), "v"(av[3]));
}

// ---- edge backward (basic.py:107-144, 167-173 reversed) ----------------------------------------
// One kernel per layer does the per-edge reverse pass AND the edge-level weight gradients: each
// wave keeps dW2 = sum_e gz2 (x) a and dWc1 = sum_e gz3 (x) m in MFMA accumulators (plus the bias,
// coord-output and scalar-input-column sums in per-lane registers) and writes one partial per wave;
// gemm_reduce adds the partials in a fixed order (deterministic). No per-edge operand ever goes to
// HBM (the unfused version wrote 6 x 64 floats per edge, 3 GB per layer at C2).
//
// Weight-gradient MFMA (wgrad_h16): fp16x3 v_mfma_f32_16x16x16_f16 with K = the unit's 16 edges. The
// ECL holds edges along lane & 15, so a unit's [16 edges][64] operands go through a per-wave LDS tile
// ([edge][ROWT]) and come back with channels along lane & 15: lane (e', g) reads edges 4g .. 4g + 3,
// channel 16t + e' (row stride 68 floats: the two 32-lane halves of a ds_read_b32 and the 8-lane
// groups of a ds_write_b128 hit distinct banks). The W1 scalar-input columns' gradient is summed per
// lane on the VALU (accFe) and across the lane group's edges once at the end.
//
// Per-wave partial (floats), blocks in gemm_reduce's [M][N+1] layout (column N = bias):
constexpr int EW_W2 = 0;                  // dW2  [64][65], column 64 = db2
constexpr int EW_WC1 = 64 * 65;           // dWc1 [64][65], column 64 = dbc1
constexpr int EW_WC2 = 2 * 64 * 65;       // dwc2 [1][65],  column 64 = dbc2
constexpr int EW_FEAT = EW_WC2 + 68;      // dW1 scalar-input columns [64][NF + 1] (NF = 1 + ne <= 5)
constexpr int EW_STRIDE = EW_FEAT + 64 * 6;
constexpr int EB_MAX_BLOCKS = 256;        // edge_bwd grid cap: EB_MAX_BLOCKS * 4 wave partials
constexpr int EB_N_MAX = 115;             // largest N whose pass A tables fit at one tile per chunk (2N senders)
constexpr int ROWT = 68;                  // transpose-tile row stride (floats)
constexpr int EB_TSTRIDE = 2 * 16 * ROWT; // per-wave transpose tile (two [16][ROWT] operands)

struct EdgeBwdArgs {
  int n_graphs, N, ne, ef_mod, ct, s_max;
  int gtab;    // pass B with the sender sums GB / GX added straight into HBM (float atomics) instead of
               // wave-private LDS tables: the large-N form (the tables' 4 x s_max rows do not fit)
  int segno;   // SEGNO_GCL (gcl.py:97-100): every edge's translation r c is clamped to +-100 before the
               // mean, so its gradient passes only where |r_d c| <= 100 (EGNO clamps the mean instead)
  const float* h; const float* x; const float* ef; const float* bb;
  const float* gF; const float* gM;
  float* GA; float* GB; float* GX;                                    // per node (GB, GX atomically)
  float* wpart;                                                       // [grid * 4][EW_STRIDE]
  // pass A -> pass B handoff of gz2 = dL/dz2 and the coordinate-MLP output c per edge: the unit
  // (tile at row rt of block b, sender offset k) owns the 16-row block (k - 1)(n + 16 G) + rt + 16 b
  // (16 x 64 floats of stash, channel-block-major so each store instruction writes 1 KB contiguous;
  // 16 floats of stash_c). The 16 b shift keeps a block's partial last tile off the next block's rows.
  float* stash; float* stash_c;
  // per node: P = W_A h + b1 and Q = W_B h, written by pass A for its chunks' receiver rows (each node
  // is a receiver of exactly one chunk) and copied into pass B's tables (no second projection)
  float* Pn; float* Qn;
};

// PASS 1 sums GA (per receiver), GB (per sender) and GX in WAVE-PRIVATE LDS tables by plain
// read-add-write (the 16 receivers and the 16 senders of one unit are distinct, and one wave's
// units run in order), and the four tables are added at the end of the chunk: LDS float atomics
// (ds_add_f32, 38 per unit) had cost more than the whole rest of the pass.
constexpr int EB_VSTAGE = BOFF_SCAL + 64 - BOFF_FEAT;   // feature k-steps + vectors + scalars
// staged fp16 hi/lo fragments: pass A W2, Wc1, Wc1^T (+ EB_VSTAGE), pass B W2^T
constexpr int EB_HSTAGE_A = 3 * 4096, EB_HSTAGE_B = 4096;
size_t edge_bwd_lds_floats(int pass, int ct, int N, int* s_max_out, int gtab = 0) {
  const int s_max = ((16 * ct - 1) / N + 2) * N;
  if (s_max_out) *s_max_out = s_max;
  // sP, sGM [ct*16][ROWP]; sQ [s_max][ROWP]; sX [s_max][4]; sGF [ct*16][4]; 4 x tile;
  // PASS 1: 4 x (sGA [ct*16][ROWP], sGB [s_max][ROWP], sGX [s_max][4]); gtab: 4 x sGA only
  // + the fp16 hi/lo fragment sets staged once
  return (pass ? EB_HSTAGE_B : EB_HSTAGE_A + EB_VSTAGE) + (size_t)ct * 16 * ROWP * (pass ? 1 : 2) + (size_t)s_max * ROWP + (size_t)s_max * 4 + (size_t)ct * 16 * 4 +
         4 * (size_t)EB_TSTRIDE + (pass ? 4 * ((size_t)ct * 16 * ROWP + (gtab ? 0 : (size_t)s_max * (ROWP + 4))) : 0);
}

// acc[ot][it] += sum over the unit's 16 edges of G[e] (x) A[e], accumulated in image-column order
// (chan_img, below: the order of the pair path's K = 32 form, so both forms share one accumulator):
// lane (e, g) of acc[ot][it][q] holds dW[chan_img(ot, 4g + q)][chan_img(it, e)].
// fp16x3 on v_mfma_f32_16x16x16_f16 (K = the unit's 16 edges: lane (e', g) supplies edges
// 4g .. 4g+3 of channel chan_img(t, e') after the LDS transpose). acc is kept in units of 1/sc: sc is
// a wave-uniform running power-of-two scale for G, lowered (and acc rescaled, exactly) when a unit's G
// is larger than any before it, so G sc stays below 2^12. The bias gradient (sum of G) is summed
// unscaled in ECL registers by the caller.
// exact: A beyond the fp16 range (a diverged rollout) -> the f32 MFMA form for this unit.
// max |x| over a lane's 16 values as a tree (v_max3), not a 16-long dependent chain
// channel held by image column 16 t + i (see the pair path below)
__device__ __forceinline__ int chan_img(int t, int i) {
  const int s = t >> 1, g = 2 * (t & 1) + (i >> 3), j = i & 7;
  return 16 * (2 * s + (j >> 2)) + 4 * g + (j & 3);
}
// running-scale update shared by both weight-gradient forms: cm = col_max of this step's G
__device__ __forceinline__ void wgrad_rescale(f4 (&acc)[4][4], float& sc, float cm, float* bsum = nullptr) {
  const float m = row_max16(cm);
  const float mu = __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, m)));
  if (mu > 0.f) {
    const float su = p2scale(mu);
    if (su < sc) {
      const float r = su / sc;
#pragma unroll
      for (int ot = 0; ot < 4; ++ot) {
        if (bsum) bsum[ot] *= r;
#pragma unroll
        for (int it = 0; it < 4; ++it) acc[ot][it] *= r;
      }
      sc = su;
    }
  }
}
// cm: col_max(amax16(G)), shared with the transposed product of the same G (mm64_cs)
// AG: the accumulators live in AGPRs, in image-column order (the pair path's form, whose asm blocks
// these use); else builtins in natural channel order (column 16 t + e), with the bias sum of G taken
// here: bsum[t] += G summed over the lane's four edges at channel 16 t + e, in units of 1/sc (round 3's
// form, which the single-unit-only pass keeps)
template <bool AG>
__device__ __forceinline__ void wgrad_h16(f4 (&acc)[4][4], float& sc, const f4 (&G)[4], const f4 (&A)[4],
                                          float* tile, int g, int e, bool exact, float cm, float (&bsum)[4]) {
  // G goes to the transpose tile unscaled, so the wave-wide max / scale below runs beside the LDS
  // round trip instead of before it; the scale is applied to the transposed values
  float* tG = tile;
  float* tA = tile + 16 * ROWT;
  store_ecl(tG + e * ROWT, G, g);
  store_ecl(tA + e * ROWT, A, g);
  wgrad_rescale(acc, sc, cm, AG ? nullptr : bsum);
  __builtin_amdgcn_wave_barrier();
  int ce[4];   // this lane's channel of column 16 t + e
#pragma unroll
  for (int t = 0; t < 4; ++t) ce[t] = AG ? chan_img(t, e) : 16 * t + e;
  if (__builtin_expect(exact, 0)) {
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const int row = (4 * g + ks) * ROWT;
      float gv[4], av[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        gv[t] = tG[row + ce[t]] * sc;
        av[t] = tA[row + ce[t]];
        if constexpr (!AG) bsum[t] += gv[t];
      }
      if constexpr (AG) {
        amfma4_block(acc, gv, av);
      } else {
#pragma unroll
        for (int ot = 0; ot < 4; ++ot)
#pragma unroll
          for (int it = 0; it < 4; ++it) acc[ot][it] = mfma(gv[ot], av[it], acc[ot][it]);
      }
    }
    __builtin_amdgcn_wave_barrier();
    return;
  }
  // A columns once (16 VGPRs of halves), G streamed one output tile at a time
  h4 ah[4], al[4];
#pragma unroll
  for (int it = 0; it < 4; ++it) {
    f4 v;
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) v[ks] = tA[(4 * g + ks) * ROWT + ce[it]];
    h4_split(v, ah[it], al[it]);
  }
#pragma unroll
  for (int ot = 0; ot < 4; ++ot) {
    f4 v;
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) v[ks] = tG[(4 * g + ks) * ROWT + ce[ot]] * sc;
    if constexpr (!AG) bsum[ot] += (v[0] + v[1]) + (v[2] + v[3]);
    h4 gh, gl;
    h4_split(v, gh, gl);
    if constexpr (AG) {
      amfma16_block(acc[ot], gl, gh, ah, al);   // G_lo A_hi + G_hi A_lo + G_hi A_hi
    } else {
#pragma unroll
      for (int it = 0; it < 4; ++it) {
        acc[ot][it] = mfma16k16(gl, ah[it], acc[ot][it]);
        acc[ot][it] = mfma16k16(gh, al[it], acc[ot][it]);
        acc[ot][it] = mfma16k16(gh, ah[it], acc[ot][it]);
      }
    }
  }
  __builtin_amdgcn_wave_barrier();
}

// ---- two units at a time (pair path): K = 32 weight-gradient MFMAs from fp16 LDS images ----------
// A pair's two 16-edge units are the 32 rows (edges) of an fp16 image [edge][64 channels], one image for
// the hi and one for the lo parts (4 KB each, per wave). Lane (e, g) writes the 8 halves of its h8
// hi[s] / lo[s] split (channels 16 (2s + (j >> 2)) + 4g + (j & 3), j = 0..7) as one 16-byte chunk at
// image column 32s + 8g: image column 16t + i therefore holds channel chan_img(t, i) below. The tile is
// read back transposed with ds_read_b64_tr_b16 (16 lanes: 4 edges x 16 image columns, column i to lane
// i), which gives the K = 32 operands of v_mfma_f32_16x16x32_f16 directly: lane l supplies edges
// 8 (l >> 4) .. + 7 of image column 16t + (l & 15). The weight gradient is therefore accumulated in
// image-column order on both axes and un-permuted when it is written out (put_pair).
// Chunks are XOR-swizzled per row (chunk ^ img_swz(row)): conflict-free transposed reads and 2-way
// b128 writes (the minimum for 16 lanes x 16 bytes on 32 banks).
// lane (e, g) writes its split of unit `u` (rows 16 u + e)
__device__ __forceinline__ void img_put(_Float16* hi_img, _Float16* lo_img, const h8 (&hi)[2], const h8 (&lo)[2],
                                        int u, int e, int g) {
  const int r = 16 * u + e;
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    *reinterpret_cast<h8*>(hi_img + img_off(r, 4 * s + g)) = hi[s];
    *reinterpret_cast<h8*>(lo_img + img_off(r, 4 * s + g)) = lo[s];
  }
}
// accP[ot][it] += sum over the pair's 32 edges of G[e] (x) A[e] in image-column order (lane (i, g) of
// accP[ot][it][q] = dW[chan_img(ot, 4g + q)][chan_img(it, i)]), fp16x3 on v_mfma_f32_16x16x32_f16.
// A: the pair's activations, already split (the forward product's split); G: the pair's gradients,
// multiplied by the wave-uniform running scale sc here and split. img: this wave's 8 KB (hi | lo).
__device__ __forceinline__ void wgrad_pair(f4 (&acc)[4][4], float& sc, const f4 (&G0)[4], const f4 (&G1)[4],
                                           const h8 (&a0h)[2], const h8 (&a0l)[2], const h8 (&a1h)[2],
                                           const h8 (&a1l)[2], _Float16* img, int e, int g, int lane, float cm) {
  _Float16* ih = img;
  _Float16* il = img + IMG_HALVES;
  img_put(ih, il, a0h, a0l, 0, e, g);
  img_put(ih, il, a1h, a1l, 1, e, g);
  // wave-uniform running scale (as wgrad_h16): cm is the larger of the two units' column maxima
  wgrad_rescale(acc, sc, cm);
  __builtin_amdgcn_wave_barrier();
  h8 bh[4], bl[4];   // B operand (activations) fragments, image columns 16 it + (lane & 15)
#pragma unroll
  for (int it = 0; it < 4; ++it) { bh[it] = tr_read8(ih, it, lane); bl[it] = tr_read8(il, it, lane); }
  // the G image overwrites the A image: every lane's A reads were issued before (LDS is in order per wave)
  __builtin_amdgcn_wave_barrier();
  {
    f4 gs[4];
    h8 gh[2], gl[2];
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) gs[mt] = G0[mt] * sc;
    h16_split(gs, gh, gl);
    img_put(ih, il, gh, gl, 0, e, g);
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) gs[mt] = G1[mt] * sc;
    h16_split(gs, gh, gl);
    img_put(ih, il, gh, gl, 1, e, g);
  }
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int ot = 0; ot < 4; ++ot) {
    const h8 ah = tr_read8(ih, ot, lane), al = tr_read8(il, ot, lane);
    amfma32_block(acc[ot], al, ah, bh, bl);   // G_lo A_hi + G_hi A_lo + G_hi A_hi
  }
  __builtin_amdgcn_wave_barrier();
}
// out0/1 += W x0/1 for two gradient column sets, each column scaled to [2^11, 2^12) before the split
// (mm64_cs for two units sharing the fragment reads)
__device__ __forceinline__ void mm64_cs2(f4 (&out0)[4], f4 (&out1)[4], const h8* wh, const f4 (&x0)[4],
                                         const f4 (&x1)[4], int lane, unsigned us, float cm0, float cm1) {
  const float sc0 = p2scale(cm0), sc1 = p2scale(cm1);
  const float inv0 = 1.f / sc0, inv1 = 1.f / sc1;   // exact (powers of two)
  f4 xs[4], acc0[4], acc1[4];
  h8 x0h[2], x0l[2], x1h[2], x1l[2];
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) { xs[mt] = x0[mt] * sc0; acc0[mt] = f4{0.f, 0.f, 0.f, 0.f}; }
  h16_split(xs, x0h, x0l);
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) { xs[mt] = x1[mt] * sc1; acc1[mt] = f4{0.f, 0.f, 0.f, 0.f}; }
  h16_split(xs, x1h, x1l);
  mfma_h16x2(acc0, acc1, wh, x0h, x0l, x1h, x1l, lane, us);
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) { out0[mt] += acc0[mt] * inv0; out1[mt] += acc1[mt] * inv1; }
}

// dst[o] = sum of the block's four wave partials (LDS, EW_STRIDE apart) for o in [o0, o1)
__device__ __forceinline__ void block_partial(const float* red, float* dst, int o0, int o1) {
  __syncthreads();
  for (int o = o0 + (int)threadIdx.x; o < o1; o += 256)
    dst[o] = ((red[o] + red[EW_STRIDE + o]) + red[2 * EW_STRIDE + o]) + red[3 * EW_STRIDE + o];
}

// sum over the 16 lanes of a lane group (the edges of a unit)
__device__ __forceinline__ float edge_sum16(float v) {
#pragma unroll
  for (int o = 1; o < 16; o <<= 1) v += __shfl_xor(v, o);
  return v;
}

// Two launches per layer (register budget: one wave cannot hold both 64x64 accumulators next to the
// per-edge working set). PASS 0 (pass A) recomputes the edge forward, accumulates dWc1, dbc1, dwc2,
// dbc2 and hands gz2 = dL/dz2 and c to pass B through HBM (stash); PASS 1 (pass B) recomputes only
// z1 and does the rest of the reverse: dW2, db2, W2^T, the W1 scalar columns and GA / GB / GX.
// OPT: 1 = EGNO norm=True (radial input normalised, basic.py:140-141), 2 = SEGNO tanh=True (coordinate
// output through tanh, gcl.py:57-59); each its own copy of the body (no per-edge select by default)
// GT: pass B's sender sums, 0 = LDS tables, 1 = HBM atomics (EdgeBwdArgs::gtab, large N), 2 = read gtab
// (the option variants); each its own copy for OPT 0 / 3, so the default loop carries no gtab branch
template <int NE, int PASS, int OPT, int GT>
__device__ __forceinline__ void edge_bwd_body(const EdgeBwdArgs& p) {
  constexpr bool rnorm = OPT == 1, ctanh = OPT == 2;
  [[maybe_unused]] constexpr bool stamp_here = OPT == 0 && GT == 0;   // (NONODE_STAMP builds)
  const bool gtab = PASS == 1 && (GT == 2 ? p.gtab != 0 : GT == 1);
  // OPT 0: EGNO, OPT 3: SEGNO (compile-time: no per-edge branch); the option variants read p.segno
  const bool segno = OPT == 0 ? false : (OPT == 3 ? true : p.segno != 0);
  extern __shared__ __attribute__((aligned(16))) float smem[];
  constexpr int NW = 4;
  constexpr int NF = 1 + NE;   // scalar inputs of edge W1: |r|^2, e_0 .. e_{NE-1}
  // two units per iteration (the pair loops below; else one unit at a time throughout)
  // pass A runs two units per iteration; pass B's pair form measured slower
  // (round 4: 524 -> 664 us per C4 layer with the handoff prefetched, 581 without; both spill) and was
  // removed
  constexpr bool PAIRS = PASS == 0;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, e = lane & 15, g = lane >> 4;
  const int N = p.N, Nm1 = N - 1;
  const int rows = p.ct * 16;
  // LDS-staged fragments: PASS 0 the forward W2, Wc1 (used twice per unit there), PASS 1 W2^T, Wc1^T
  float* sH = smem;
  float* sP = smem + (PASS ? EB_HSTAGE_B : EB_HSTAGE_A + EB_VSTAGE);
  float* sGM = sP + rows * ROWP;   // pass A only
  float* sQ = PASS ? sGM : sGM + rows * ROWP;
  float* sX = sQ + p.s_max * ROWP;
  float* sGF = sX + p.s_max * 4;
  float* tile = sGF + rows * 4 + wave * EB_TSTRIDE;
  float* sGA = sGF + rows * 4 + NW * EB_TSTRIDE;   // [NW][rows][ROWP]     (PASS 1)
  float* sGB = sGA + NW * rows * ROWP;              // [NW][s_max][ROWP]
  float* sGX = sGB + NW * p.s_max * ROWP;           // [NW][s_max][4]
  float* myGA = sGA + wave * rows * ROWP;
  float* myGB = sGB + wave * p.s_max * ROWP;
  float* myGX = sGX + wave * p.s_max * 4;
  const float* bb = p.bb;
  const float bc2 = bb[BOFF_SCAL + 0];
  const float* wW2 = bb + BOFF_W2;
  const float* wWc1 = bb + BOFF_WC1;
  {
    // pass A: W2 | Wc1 (adjacent in the blob) and Wc1^T; pass B: W2^T
    const f4* src = reinterpret_cast<const f4*>(bb + BOFF_H16 + (PASS == 0 ? BH_W2 : BH_W2T) * 4096);
    for (int i = tid; i < (PASS == 0 ? 2 : 1) * 1024; i += NW * 64) reinterpret_cast<f4*>(sH)[i] = src[i];
    if (PASS == 0) {
      const f4* srcT = reinterpret_cast<const f4*>(bb + BOFF_H16 + BH_WC1T * 4096);
      for (int i = tid; i < 1024; i += NW * 64) reinterpret_cast<f4*>(sH + 8192)[i] = srcT[i];
      const f4* vsrc = reinterpret_cast<const f4*>(bb + BOFF_FEAT);
      for (int i = tid; i < EB_VSTAGE / 4; i += NW * 64) reinterpret_cast<f4*>(sH + EB_HSTAGE_A)[i] = vsrc[i];
    }
  }
  const float* sV = PASS == 0 ? sH + EB_HSTAGE_A : bb + BOFF_FEAT;   // bb + BOFF_FEAT .. BOFF_SCAL + 64
  const h8* hW2 = PASS == 0 ? reinterpret_cast<const h8*>(sH) : reinterpret_cast<const h8*>(bb + BOFF_H16 + BH_W2 * 4096);
  const h8* hWc1 = PASS == 0 ? reinterpret_cast<const h8*>(sH + 4096) : reinterpret_cast<const h8*>(bb + BOFF_H16 + BH_WC1 * 4096);
  const h8* hW2T = reinterpret_cast<const h8*>(sH);
  const h8* hWc1T = reinterpret_cast<const h8*>(sH + 8192);   // pass A only
  float scW = 0x1p112f;   // running scale of the accW / sB sums (wgrad_h16)
  f4 accW[4][4];   // PASS 0: dWc1 (AGPRs in the pair path: amfma32_block), PASS 1: dW2
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) accW[a][b] = f4{0.f, 0.f, 0.f, 0.f};
  // pass B: dW1 scalar-input columns per lane, sum over the lane's edges of fe[f] gz1 (the 16 edges
  // of a lane group are added once at the end): NF x 16 FMAs per unit on the VALU instead of a
  // transpose through LDS and 16 f32 MFMAs
  f4 accFe[NF][4], sWC2[4];
#pragma unroll
  for (int f = 0; f < NF; ++f) zero4(accFe[f]);
  zero4(sWC2);
  // bias gradient (PASS 0: dbc1, PASS 1: db2): with the pair path per lane in ECL (bsE, summed over the
  // lane group's edges at the end), else per lane at channel 16 t + e in units of 1/scW (sB, wgrad_h16)
  f4 bsE[4];
  zero4(bsE);
  float sB[4] = {0.f, 0.f, 0.f, 0.f};
  float sGC = 0.f;
  const int G = gridDim.x;
  const int nb = (int)(((long long)blockIdx.x * p.n_graphs) / G) * N;
  const int nend = (int)(((long long)(blockIdx.x + 1) * p.n_graphs) / G) * N;
  const int ntw = (nend - nb + 15) >> 4;
  const int nch = (ntw + p.ct - 1) / p.ct;
  STAMP_DECL   // diagnostic section stamps (NONODE_STAMP builds): PASS 1 slots 0-12, PASS 0 13-15
  // chunk ci: ctc tiles from row rbase; its senders are the S rows of the graphs it touches, from s0
  struct Chunk { int ctc, rbase, s0, S; };
  auto chunk_at = [&](int ci) __attribute__((always_inline)) {
    Chunk c;
    const int c0 = (ci * ntw) / nch;
    c.ctc = ((ci + 1) * ntw) / nch - c0;
    c.rbase = nb + c0 * 16;
    const int r_last = min(c.rbase + c.ctc * 16, nend) - 1;
    const int g_lo = c.rbase / N, g_hi = r_last / N;
    c.s0 = g_lo * N;
    c.S = (g_hi - g_lo + 1) * N;
    return c;
  };
  // The chunk's global rows (positions, gF and, in pass B, pass A's projections P / Q) are all
  // requested into registers before any is stored, and pass B's wave-private sum tables are zeroed while
  // they are in flight: one memory latency per chunk instead of one per loop trip (this phase was 17% of
  // pass B). (Requesting the next chunk's rows before this chunk's phase C instead measured no faster at
  // C4 and slower for SEGNO's small per-substep launches.)
  constexpr int KS = PASS == 1 ? 4 : 1;   // f4 rows staged per thread (ct = 1, N = 20: 896 of 1024)
  f4 st4[KS];
  float stx = 0.f, stf = 0.f;
  auto pq_at = [&](const Chunk& c, int i) __attribute__((always_inline)) {   // P of the receiver rows (zero past
    const int nP4 = c.ctc * 16 * 16;                                          // the range), Q of the senders
    if (i < nP4) {
      const int rr = c.rbase + (i >> 4);
      return rr < nend ? reinterpret_cast<const f4*>(p.Pn + (size_t)rr * HID)[i & 15] : f4{0.f, 0.f, 0.f, 0.f};
    }
    const int i2 = i - nP4;
    return reinterpret_cast<const f4*>(p.Qn + (size_t)(c.s0 + (i2 >> 4)) * HID)[i2 & 15];
  };
  auto x_at = [&](const Chunk& c, int i) __attribute__((always_inline)) {
    const int s_ = i / 3;
    return p.x[(size_t)(c.s0 + s_) * 3 + (i - 3 * s_)];
  };
  auto gf_at = [&](const Chunk& c, int i) __attribute__((always_inline)) {
    const int rr = c.rbase + i / 4;
    return rr < nend ? p.gF[(size_t)rr * 4 + (i & 3)] : 0.f;
  };
  auto stage = [&](const Chunk& c) __attribute__((always_inline)) {
    const int nT = PASS == 1 ? (c.ctc * 16 + c.S) * 16 : 0;
    stx = tid < c.S * 3 ? x_at(c, tid) : 0.f;
    stf = tid < c.ctc * 64 ? gf_at(c, tid) : 0.f;
#pragma unroll
    for (int k = 0; k < KS; ++k) {
      const int i = tid + k * NW * 64;
      if (i < nT) st4[k] = pq_at(c, i);
    }
  };
  for (int ci = 0; ci < nch; ++ci) {
    const Chunk cc = chunk_at(ci);
    const int ctc = cc.ctc, rbase = cc.rbase, s0 = cc.s0, S = cc.S;
    const int nsT = (S + 15) >> 4;
    // ---- A: tables ----
    stage(cc);
    {
      const int nX = S * 3, nF = ctc * 16 * 4;
      const int nP4 = PASS == 1 ? ctc * 16 * 16 : 0, nT = nP4 + (PASS == 1 ? S * 16 : 0);
      auto pq_put = [&](int i, f4 v) {
        if (i < nP4) *reinterpret_cast<f4*>(sP + (i >> 4) * ROWP + 4 * (i & 15)) = v;
        else *reinterpret_cast<f4*>(sQ + ((i - nP4) >> 4) * ROWP + 4 * ((i - nP4) & 15)) = v;
      };
      if (PASS == 1) {
        const f4 z = {0.f, 0.f, 0.f, 0.f};
        for (int i = tid; i < NW * rows * ROWP / 4; i += NW * 64) reinterpret_cast<f4*>(sGA)[i] = z;
        if (!gtab)
          for (int i = tid; i < NW * p.s_max * (ROWP + 4) / 4; i += NW * 64) reinterpret_cast<f4*>(sGB)[i] = z;   // sGB, sGX
      }
      if (tid < nX) sX[(tid / 3) * 4 + tid % 3] = stx;
      if (tid < nF) sGF[tid] = stf;
#pragma unroll
      for (int k = 0; k < KS; ++k) {
        const int i = tid + k * NW * 64;
        if (i < nT) pq_put(i, st4[k]);
      }
      for (int i = tid + NW * 64; i < nX; i += NW * 64) sX[(i / 3) * 4 + i % 3] = x_at(cc, i);   // larger chunks
      for (int i = tid + NW * 64; i < nF; i += NW * 64) sGF[i] = gf_at(cc, i);
      for (int i = tid + KS * NW * 64; i < nT; i += NW * 64) pq_put(i, pq_at(cc, i));
    }
    for (int job = wave; job < (PASS == 0 ? ctc + nsT : 0); job += NW) {
      const bool isP = job < ctc;
      const int local = (isP ? job : job - ctc) * 16 + e;
      int node = isP ? rbase + local : s0 + local;
      const bool valid = isP ? (node < nend) : (local < S);
      node = valid ? node : (isP ? nend - 1 : s0);
      f4 hin[4], acc[4];
      load_ecl(hin, p.h + (size_t)node * HID, g);
      if (isP) load_vp(acc, bb + BOFF_VEC + BV_B1 * 64, g);
      else zero4(acc);
      // fp16x3 as in the forward's projections (exact f32 MFMAs beyond the fp16 range)
      if (__builtin_expect(__any(amax_ecl(hin) > H16_LIMIT), 0)) {
        mfma_dense<4>(acc, bb + (isP ? BOFF_WA : BOFF_WB), hin, lane);
      } else {
        h8 xh[2], xl[2];
        h16_split(hin, xh, xl);
        mfma_h16(acc, reinterpret_cast<const h8*>(bb + BOFF_H16 + (isP ? BH_WA : BH_WB) * 4096), xh, xl, lane,
                 h16_us(bb + BOFF_SCAL, isP ? BH_WA : BH_WB));
      }
      // rows of receivers past the range are zero: their lanes' a, m feed the weight-gradient
      // MFMAs (multiplied by zero gradients, so they must be finite)
      if (isP && !valid) zero4(acc);
      if (valid || isP) {
        store_ecl((isP ? sP : sQ) + local * ROWP, acc, g);
        // each node is a receiver of exactly one chunk: it writes that node's P and Q for pass B
        const bool mine = isP ? valid : (node >= rbase && node < rbase + ctc * 16 && node < nend);
        if (mine) store_ecl((isP ? p.Pn : p.Qn) + (size_t)node * HID, acc, g);
        if (isP) {
          f4 gm[4];
          load_ecl(gm, p.gM + (size_t)node * HID, g);
          store_ecl(sGM + local * ROWP, gm, g);
        }
      }
    }
    STAMP(PASS ? 8 : 14);
    __syncthreads();
    STAMP(PASS ? 9 : 14);
    // ---- B: one unit (16 edges: receivers of a tile x sender offset k) at a time ----
    const int U = ctc * Nm1;
    f4 gaR[4];   // pass B: GA of the current tile's receivers (lane e), and the receiver-side GX
    zero4(gaR);
    float gxR0 = 0.f, gxR1 = 0.f, gxR2 = 0.f;
    int cur_tau = -1;
    auto flush_ga = [&](int t) {   // into the wave-private tables (distinct receivers: no race)
      const int rl_ = 16 * t + e;
      f4 v[4];
      load_ecl(v, myGA + rl_ * ROWP, g);
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) v[mt] += gaR[mt];
      store_ecl(myGA + rl_ * ROWP, v, g);
      const int rr = rbase + rl_;
      if (g == 0 && rr < nend) {
        if (gtab) {   // large N: no sender tables, the receiver side joins the HBM sums too
          atomicAdd(p.GX + (size_t)rr * 4 + 0, gxR0);
          atomicAdd(p.GX + (size_t)rr * 4 + 1, gxR1);
          atomicAdd(p.GX + (size_t)rr * 4 + 2, gxR2);
        } else {
          f4* xr = reinterpret_cast<f4*>(myGX + (rr - s0) * 4);
          *xr += f4{gxR0, gxR1, gxR2, 0.f};
        }
      }
      zero4(gaR);
      gxR0 = gxR1 = gxR2 = 0.f;
    };
    // a lane's receiver geometry in tile tau (one integer division per tile, not per unit): row rl in
    // the chunk, in range, graph-local index n, the graph's first row in the sender table, edge rows
    struct LT { int tau, rl, n, sb; bool rv; size_t efb; };
    auto lane_tile = [&](int tau) __attribute__((always_inline)) {
      LT t;
      t.tau = tau;
      t.rl = 16 * tau + e;
      const int r = rbase + t.rl;
      t.rv = r < nend;
      const int rc = t.rv ? r : nend - 1;
      const int gr = rc / N;
      t.n = rc - gr * N;
      t.sb = gr * N - s0;
      t.efb = ((size_t)(gr % p.ef_mod) * N + t.n) * Nm1;
      return t;
    };
    // unit u = tau (N - 1) + k - 1 of the chunk, stepped without a division
    auto unit_tk = [&](int u, int& tau, int& k) __attribute__((always_inline)) {
      tau = u / Nm1;
      k = u - tau * Nm1 + 1;
    };
    auto step_tk = [&](int& tau, int& k, int by) __attribute__((always_inline)) {
      k += by;
      while (k > Nm1) { k -= Nm1; ++tau; }
    };
    // the wave's next unit's edge features and (pass B) handoff block are requested one unit ahead,
    // so their global-memory latency overlaps this unit's work
    auto unit_src = [&](const LT& t, int k_, const float*& efp_o, size_t& sunit_o) __attribute__((always_inline)) {
      int j_ = t.n + k_;
      j_ = (j_ >= N) ? j_ - N : j_;
      const int jj_ = (j_ < t.n) ? j_ : j_ - 1;
      efp_o = p.ef + (t.efb + jj_) * NE;
      sunit_o = (size_t)(k_ - 1) * ((size_t)p.n_graphs * N + 16 * gridDim.x) + rbase + 16 * t.tau + 16 * blockIdx.x;
    };
    float efn[NE > 0 ? NE : 1];
    f4 gzn[4];
    float cn = 0.f;
    auto prefetch = [&](const LT& t, int k_) __attribute__((always_inline)) {
      const float* ep;
      size_t su;
      unit_src(t, k_, ep, su);
#pragma unroll
      for (int kk = 0; kk < NE; ++kk) efn[kk] = ep[kk];
      if constexpr (PASS == 1) {
        const float* sb16 = p.stash + su * HID;
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) gzn[mt] = *reinterpret_cast<const f4*>(sb16 + mt * 256 + e * 16 + 4 * g);
        cn = p.stash_c[su + e];
      }
    };
    constexpr int NEP = NE > 0 ? NE : 1;
    // one unit (16 edges) through the whole reverse pass of this PASS (the single-unit form: every
    // unit of pass B, pass A's odd last unit and its pairs whose activations leave the fp16 range)
    auto unit_one = [&](const LT& lt, int k, const float (&fe_in)[NEP], const f4 (&gz_in)[4], float c_in) __attribute__((always_inline)) {
      const int tau = lt.tau, rl = lt.rl, n = lt.n, sb = lt.sb;
      const bool rvalid = lt.rv;
      int j = n + k;
      j = (j >= N) ? j - N : j;
      const int sl = sb + j, rls = sb + n;
      const float r0 = sX[rls * 4 + 0] - sX[sl * 4 + 0];
      const float r1 = sX[rls * 4 + 1] - sX[sl * 4 + 1];
      const float r2 = sX[rls * 4 + 2] - sX[sl * 4 + 2];
      const float s2 = fmaf(r0, r0, fmaf(r1, r1, r2 * r2));
      float fe[NF];
      fe[0] = s2;
      if constexpr (rnorm) fe[0] = radial_norm(s2);
#pragma unroll
      for (int kk = 0; kk < NE; ++kk) fe[1 + kk] = fe_in[kk];
      float ev[2];
#pragma unroll
      for (int kf = 0; kf < 2; ++kf) {
        const int fi = 4 * kf + g;
        ev[kf] = 0.f;
#pragma unroll
        for (int kk = 0; kk < NF; ++kk) ev[kf] = (fi == kk) ? fe[kk] : ev[kf];
      }
      // forward recompute: z1 = P_r + Q_s + W1[:, s|e] [s, e];  a = SiLU(z1)
      f4 z1[4], q4[4];
      load_ecl(z1, sP + rl * ROWP, g);
      load_ecl(q4, sQ + sl * ROWP, g);
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) z1[mt] += q4[mt];
#pragma unroll
      for (int kf = 0; kf < 2; ++kf) {
        if (kf * 4 < NF) {
          const f4 wf = *reinterpret_cast<const f4*>(sV + kf * 256 + lane * 4);
#pragma unroll
          for (int mo = 0; mo < 4; ++mo) z1[mo] = mfma(wf[mo], ev[kf], z1[mo]);
        }
      }
      // this unit's handoff block: 16 edges x 64 channels, contiguous (stash_at)
      const size_t sunit = (size_t)(k - 1) * ((size_t)p.n_graphs * N + 16 * gridDim.x) + rbase + 16 * tau + 16 * blockIdx.x;
      f4 sg1[4], gz2[4];
      bool bigA;
      float c;
      if constexpr (PASS == 0) {
        // a = SiLU(z1); z2 = W2 a + b2; m = SiLU(z2); z3 = Wc1 m + bc1; c1 = SiLU(z3) (fp16x3 on the
        // matrix cores, exact f32 MFMAs for a unit whose activations leave the fp16 range)
        f4 z2[4], sg2[4], z3[4], sg3[4];
        bool bigM;
        {
          // fp16x3 unconditionally, so silu -> W2 -> silu -> Wc1 is one basic block for the scheduler;
          // a unit whose activations leave the fp16 range is recomputed afterwards with exact f32
          // MFMAs (both products; its dWc1 term then takes the exact form too)
          STAMP(13);   // pass A sections: 13 head, 2 forward W2 / Wc1 / c, 15 gz3 + dWc1, 3 Wc1^T, 4 handoff
          float ma, mm;
          {
            f4 a[4];
            silu_keep(z1, sg1, a);
            ma = amax16(a);
            load_vp(z2, sV + (BOFF_VEC - BOFF_FEAT) + BV_B2 * 64, g);
            h8 xh[2], xl[2];
            h16_split(a, xh, xl);
            mfma_h16(z2, hW2, xh, xl, lane, h16_us(bb + BOFF_SCAL, BH_W2));
          }
          {
            f4 m[4];
            silu_keep(z2, sg2, m);
            mm = amax16(m);
            load_vp(z3, sV + (BOFF_VEC - BOFF_FEAT) + BV_BC1 * 64, g);
            h8 xh[2], xl[2];
            h16_split(m, xh, xl);
            mfma_h16(z3, hWc1, xh, xl, lane, h16_us(bb + BOFF_SCAL, BH_WC1));
          }
          bigA = __any(ma > H16_LIMIT);
          bigM = __any(mm > H16_LIMIT);
          if (__builtin_expect(bigA || bigM, 0)) {
            f4 a[4], m[4];
#pragma unroll
            for (int mt = 0; mt < 4; ++mt) a[mt] = z1[mt] * sg1[mt];
            load_vp(z2, sV + (BOFF_VEC - BOFF_FEAT) + BV_B2 * 64, g);
            mfma_dense<4>(z2, wW2, a, lane);
            silu_keep(z2, sg2, m);
            load_vp(z3, sV + (BOFF_VEC - BOFF_FEAT) + BV_BC1 * 64, g);
            mfma_dense<4>(z3, wWc1, m, lane);
            bigM = true;
          }
        }
        {
          f4 c1[4];
          silu_keep(z3, sg3, c1);
          c = dot_vp(c1, sV + (BOFF_VEC - BOFF_FEAT) + BV_WC2 * 64, g) + bc2;
          if constexpr (ctanh) c = tanhf(c);
        }
        STAMP(2);
        // reverse: f = r c (SEGNO: clamp(r c, +-100) per edge)
        float gF0 = sGF[rl * 4 + 0], gF1 = sGF[rl * 4 + 1], gF2 = sGF[rl * 4 + 2];
        if (segno) {
          gF0 = fabsf(r0 * c) <= 100.f ? gF0 : 0.f;
          gF1 = fabsf(r1 * c) <= 100.f ? gF1 : 0.f;
          gF2 = fabsf(r2 * c) <= 100.f ? gF2 : 0.f;
        }
        float gc = rvalid ? (gF0 * r0 + gF1 * r1 + gF2 * r2) : 0.f;
        if constexpr (ctanh) gc *= 1.f - c * c;   // through the tanh: gc is the gradient of the MLP output
        // c = wc2 . c1 + bc2 ; c1 = SiLU(z3)
        f4 gz3[4];
        load_vp(gz3, sV + (BOFF_VEC - BOFF_FEAT) + BV_WC2 * 64, g);
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) gz3[mt] *= gc;
        mul_dsilu_s(gz3, z3, sg3);
        // dWc1 += gz3 (x) m ; dwc2 += gc c1 ; dbc1 += gz3 ; dbc2 += gc
        const float cm3 = col_max(amax16(gz3));
        {
          f4 m[4];
#pragma unroll
          for (int mt = 0; mt < 4; ++mt) m[mt] = z2[mt] * sg2[mt];
          wgrad_h16<PAIRS>(accW, scW, gz3, m, tile, g, e, bigM, cm3, sB);
          if constexpr (PAIRS) {
#pragma unroll
            for (int mt = 0; mt < 4; ++mt) bsE[mt] += gz3[mt];
          }
        }
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) sWC2[mt] += gc * (z3[mt] * sg3[mt]);
        sGC += gc;
        STAMP(15);
        // z3 = Wc1 m + bc1: gm = Wc1^T gz3 + gM_r (M = sum_j m); gz2 = gm SiLU'(z2) -> pass B
        load_ecl(gz2, sGM + rl * ROWP, g);
        if (!rvalid) zero4(gz2);
        mm64_cs(gz2, hWc1T, gz3, lane, h16_us(bb + BOFF_SCAL, BH_WC1T), cm3);
        mul_dsilu_s(gz2, z2, sg2);                 // m = SiLU(z2)
        STAMP(3);
        // (rows past the range too: their slots lie inside this unit's block)
        {
          float* sb16 = p.stash + sunit * HID;
#pragma unroll
          for (int mt = 0; mt < 4; ++mt) *reinterpret_cast<f4*>(sb16 + mt * 256 + e * 16 + 4 * g) = gz2[mt];
          if (g == 0) p.stash_c[sunit + e] = c;
        }
        STAMP(4);
        return;
      } else {
        f4 a[4];
        STAMP(0);
        silu_keep(z1, sg1, a);
        bigA = __any(amax_ecl(a) > H16_LIMIT);
        // pass A's gz2 and c of this edge (zero gradient for receivers past the range)
        c = c_in;
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) gz2[mt] = gz_in[mt];
        if (!rvalid) zero4(gz2);
      }
      STAMP(1);
      float gF0 = sGF[rl * 4 + 0], gF1 = sGF[rl * 4 + 1], gF2 = sGF[rl * 4 + 2];
      if (segno) {
        gF0 = fabsf(r0 * c) <= 100.f ? gF0 : 0.f;
        gF1 = fabsf(r1 * c) <= 100.f ? gF1 : 0.f;
        gF2 = fabsf(r2 * c) <= 100.f ? gF2 : 0.f;
      }
      float gr0 = c * gF0, gr1 = c * gF1, gr2 = c * gF2;
      // dW2 += gz2 (x) a ; db2 += gz2
      const float cm2 = col_max(amax16(gz2));
      {
        f4 a[4];
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) a[mt] = z1[mt] * sg1[mt];
        wgrad_h16<PAIRS>(accW, scW, gz2, a, tile, g, e, bigA, cm2, sB);
        if constexpr (PAIRS) {
#pragma unroll
          for (int mt = 0; mt < 4; ++mt) bsE[mt] += gz2[mt];
        }
      }
      STAMP(5);
      f4 gz1[4];
      zero4(gz1);
      mm64_cs(gz1, hW2T, gz2, lane, h16_us(bb + BOFF_SCAL, BH_W2T), cm2);
      STAMP(6);
      mul_dsilu_s(gz1, z1, sg1);                 // a = SiLU(z1)
      // scalar-input columns of W1: dW1[:, f] += gz1 (x) fe[f]
#pragma unroll
      for (int f = 0; f < NF; ++f)
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) accFe[f][mt] += fe[f] * gz1[mt];
      // s = |r|^2 input column
      float gs = dot_vp(gz1, sV + (BOFF_VEC - BOFF_FEAT) + BV_WS * 64, g);
      if constexpr (rnorm) gs = s2 < 1e-12f ? gs * 1e12f : 0.f;   // d normalize(s) / ds: 1 / eps below eps, else 0
      gr0 = fmaf(2.f * gs, r0, gr0);
      gr1 = fmaf(2.f * gs, r1, gr1);
      gr2 = fmaf(2.f * gs, r2, gr2);
      // GA and the receiver side of GX stay in registers while the wave's units keep the same tile
      // (a lane's receiver is fixed within a tile; lanes of rows past the range add zeros: their gz2
      // and gF are zero); the sender sums go to the wave-private tables per unit
      if (tau != cur_tau) {   // wave-uniform
        if (cur_tau >= 0) flush_ga(cur_tau);
        cur_tau = tau;
      }
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) gaR[mt] += gz1[mt];
      gxR0 += gr0;
      gxR1 += gr1;
      gxR2 += gr2;
      if (rvalid && gtab) {   // large N: straight into the (zeroed) HBM sums
        float* gb = p.GB + (size_t)(s0 + sl) * HID + 4 * g;
#pragma unroll
        for (int mt = 0; mt < 4; ++mt)
#pragma unroll
          for (int q = 0; q < 4; ++q) atomicAdd(gb + 16 * mt + q, gz1[mt][q]);
        if (g == 0) {
          float* gx = p.GX + (size_t)(s0 + sl) * 4;
          atomicAdd(gx + 0, -gr0);
          atomicAdd(gx + 1, -gr1);
          atomicAdd(gx + 2, -gr2);
        }
      } else if (rvalid) {
        f4 t[4];
        load_ecl(t, myGB + sl * ROWP, g);
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) t[mt] += gz1[mt];
        store_ecl(myGB + sl * ROWP, t, g);
        if (g == 0) {
          f4* xs = reinterpret_cast<f4*>(myGX + sl * 4);
          *xs -= f4{gr0, gr1, gr2, 0.f};
        }
      }
      STAMP(7);
    };
    // ---- shared by both passes' two-unit loops ----
    struct UnitGeo {
      int rl, sl, tau;   // receiver row (chunk), sender row (chunk tables), tile
      bool rv;           // receiver row in range
      float q0, q1, q2;  // r = x_r - x_s
      float s2;          // |r|^2
      float fe[NF];      // scalar edge inputs [|r|^2 (or its normalisation), e ...]
      size_t su;         // handoff block
    };
    auto load_ef = [&](int uu, float (&dst)[NEP]) __attribute__((always_inline)) {
      const float* ep;
      size_t su;
      int tau_, k_;
      unit_tk(uu, tau_, k_);
      unit_src(lane_tile(tau_), k_, ep, su);
#pragma unroll
      for (int kk = 0; kk < NE; ++kk) dst[kk] = ep[kk];
    };
    // z1 = P_r + Q_s + W1[:, s|e] [s, e] of unit uu, and its geometry
    auto head_u = [&](int uu, const float (&fin)[NEP], f4 (&z1)[4], UnitGeo& o) __attribute__((always_inline)) {
      const int tau = uu / Nm1, k = uu - tau * Nm1 + 1;
      const int rl = 16 * tau + e;
      const int r = rbase + rl;
      const bool rvalid = r < nend;
      const int rc = rvalid ? r : nend - 1;
      const int gr = rc / N, n = rc - gr * N;
      int j = n + k;
      j = (j >= N) ? j - N : j;
      const int sb = gr * N - s0;
      const int sl = sb + j, rls = sb + n;
      o.q0 = sX[rls * 4 + 0] - sX[sl * 4 + 0];
      o.q1 = sX[rls * 4 + 1] - sX[sl * 4 + 1];
      o.q2 = sX[rls * 4 + 2] - sX[sl * 4 + 2];
      const float s2 = fmaf(o.q0, o.q0, fmaf(o.q1, o.q1, o.q2 * o.q2));
      o.s2 = s2;
      o.fe[0] = s2;
      if constexpr (rnorm) o.fe[0] = radial_norm(s2);
#pragma unroll
      for (int kk = 0; kk < NE; ++kk) o.fe[1 + kk] = fin[kk];
      float ev[2];
#pragma unroll
      for (int kf = 0; kf < 2; ++kf) {
        const int fi = 4 * kf + g;
        ev[kf] = 0.f;
#pragma unroll
        for (int kk = 0; kk < NF; ++kk) ev[kf] = (fi == kk) ? o.fe[kk] : ev[kf];
      }
      f4 q4[4];
      load_ecl(z1, sP + rl * ROWP, g);
      load_ecl(q4, sQ + sl * ROWP, g);
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) z1[mt] += q4[mt];
#pragma unroll
      for (int kf = 0; kf < 2; ++kf) {
        if (kf * 4 < NF) {
          const f4 wf = *reinterpret_cast<const f4*>(sV + kf * 256 + lane * 4);
#pragma unroll
          for (int mo = 0; mo < 4; ++mo) z1[mo] = mfma(wf[mo], ev[kf], z1[mo]);
        }
      }
      o.rl = rl;
      o.sl = sl;
      o.tau = tau;
      o.rv = rvalid;
      o.su = (size_t)(k - 1) * ((size_t)p.n_graphs * N + 16 * gridDim.x) + rbase + 16 * tau + 16 * blockIdx.x;
    };
    // dL/dr c-part gF masked (SEGNO: the per-edge clamp passes the gradient only where |r_d c| <= 100)
    auto grad_f = [&](const UnitGeo& o, float c, float& f0, float& f1, float& f2) __attribute__((always_inline)) {
      f0 = sGF[o.rl * 4 + 0]; f1 = sGF[o.rl * 4 + 1]; f2 = sGF[o.rl * 4 + 2];
      if (segno) {
        f0 = fabsf(o.q0 * c) <= 100.f ? f0 : 0.f;
        f1 = fabsf(o.q1 * c) <= 100.f ? f1 : 0.f;
        f2 = fabsf(o.q2 * c) <= 100.f ? f2 : 0.f;
      }
    };
    // dL/dc of a unit (f = r c; tanh option)
    auto grad_c = [&](const UnitGeo& o, float c) __attribute__((always_inline)) {
      float f0, f1, f2;
      grad_f(o, c, f0, f1, f2);
      float gc = o.rv ? (f0 * o.q0 + f1 * o.q1 + f2 * o.q2) : 0.f;
      if constexpr (ctanh) gc *= 1.f - c * c;
      return gc;
    };
    int u_first = wave;
    unsigned long long bigmask = 0;   // pass A: this wave's pairs (local index) left to the single-unit form
    if constexpr (PASS == 0 && PAIRS) {
      // ---- pass A, two units per iteration: units 2i and 2i + 1 of the chunk (any two units, possibly
      // of two tiles), pair i on wave i % NW. Each LDS fragment read feeds both units' MFMAs, the
      // two dependent chains interleave, and dWc1 takes the K = 32 form (wgrad_pair) with m's split
      // from the forward Wc1 product as its operand. An odd last unit runs in the single-unit loop.
      const int npair = U >> 1;   // <= 4 * 64 pairs per chunk (ct <= 8 tiles, N <= 32): bigmask below
      u_first = ((U & 1) && wave == npair % NW) ? U - 1 : U;
      _Float16* img = reinterpret_cast<_Float16*>(tile);
      const unsigned us_w2 = h16_us(bb + BOFF_SCAL, BH_W2), us_wc1 = h16_us(bb + BOFF_SCAL, BH_WC1);
      const unsigned us_wc1t = h16_us(bb + BOFF_SCAL, BH_WC1T);
      const float* vB2 = sV + (BOFF_VEC - BOFF_FEAT) + BV_B2 * 64;
      const float* vBC1 = sV + (BOFF_VEC - BOFF_FEAT) + BV_BC1 * 64;
      const float* vWC2 = sV + (BOFF_VEC - BOFF_FEAT) + BV_WC2 * 64;
      float fa[NEP], fb[NEP];
      if (wave < npair) {
        load_ef(2 * wave, fa);
        load_ef(2 * wave + 1, fb);
      }
      for (int ip = wave; ip < npair; ip += NW) {
        asm volatile("" ::: "memory");   // keep the fragment reads in the loop (see below)
        float ea[NEP], eb[NEP];
#pragma unroll
        for (int kk = 0; kk < NEP; ++kk) { ea[kk] = fa[kk]; eb[kk] = fb[kk]; }
        {
          const int ipn = ip + NW < npair ? ip + NW : ip;
          load_ef(2 * ipn, fa);
          load_ef(2 * ipn + 1, fb);
        }
        f4 z1a[4], z1b[4];
        UnitGeo ga, gb;
        head_u(2 * ip, ea, z1a, ga);
        head_u(2 * ip + 1, eb, z1b, gb);
        STAMP(13);
        // forward recompute: a = SiLU(z1); z2 = W2 a + b2; m = SiLU(z2); z3 = Wc1 m + bc1 (fp16x3; exact
        // f32 MFMAs for a pair whose activations leave the fp16 range)
        // a = SiLU(z1) (dead after its split: the fallback below recomputes it)
        f4 z2a[4], z2b[4];
        float amx;
        {
          h8 xah[2], xal[2], xbh[2], xbl[2];
          silu_true(z1a);
          silu_true(z1b);
          amx = fmaxf(amax16(z1a), amax16(z1b));
          h16_split(z1a, xah, xal);
          h16_split(z1b, xbh, xbl);
          load_vp(z2a, vB2, g);
#pragma unroll
          for (int mt = 0; mt < 4; ++mt) z2b[mt] = z2a[mt];
          mfma_h16x2(z2a, z2b, hW2, xah, xal, xbh, xbl, lane, us_w2);
        }
        PAIR_FENCE();
        // m = SiLU(z2); d2 = SiLU'(z2) kept for gz2
        f4 d2a[4], d2b[4];
        h8 mah[2], mal[2], mbh[2], mbl[2];   // m's split: the Wc1 product's B operand and dWc1's A operand
        float mmx;
        {
          f4 ma[4], mb[4];
          silu_dsilu(z2a, ma, d2a);
          silu_dsilu(z2b, mb, d2b);
          mmx = fmaxf(amax16(ma), amax16(mb));
          h16_split(ma, mah, mal);
          h16_split(mb, mbh, mbl);
        }
        f4 z3a[4], z3b[4];
        load_vp(z3a, vBC1, g);
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) z3b[mt] = z3a[mt];
        mfma_h16x2(z3a, z3b, hWc1, mah, mal, mbh, mbl, lane, us_wc1);
        PAIR_FENCE();
        if (__builtin_expect(__any(fmaxf(amx, mmx) > H16_LIMIT), 0)) {
          // an activation beyond the fp16 range (a diverged state): the pair is redone after the loop by
          // the single-unit form, whose forward and weight gradient take exact f32 MFMAs there
          bigmask |= 1ull << ((ip - wave) / NW);
          continue;
        }
        // c1 = SiLU(z3), d3 = SiLU'(z3); c = wc2 . c1 + bc2
        f4 c1a[4], c1b[4], d3a[4], d3b[4];
        silu_dsilu(z3a, c1a, d3a);
        silu_dsilu(z3b, c1b, d3b);
        float ca = dot_vp(c1a, vWC2, g) + bc2, cb = dot_vp(c1b, vWC2, g) + bc2;
        if constexpr (ctanh) { ca = tanhf(ca); cb = tanhf(cb); }
        STAMP(2);
        // reverse: gz3 = gc wc2 SiLU'(z3); dwc2 += gc c1; dbc2 += gc; dbc1 += gz3
        const float gca = grad_c(ga, ca), gcb = grad_c(gb, cb);
        f4 gz3a[4], gz3b[4];
        load_vp(gz3a, vWC2, g);
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) {
          gz3b[mt] = gz3a[mt] * gcb * d3b[mt];
          gz3a[mt] = gz3a[mt] * gca * d3a[mt];
          sWC2[mt] += gca * c1a[mt];
          sWC2[mt] += gcb * c1b[mt];
          bsE[mt] += gz3a[mt];
          bsE[mt] += gz3b[mt];
        }
        sGC += gca;
        sGC += gcb;
        const float cma = col_max(amax16(gz3a)), cmb = col_max(amax16(gz3b));
        // dWc1 += gz3 (x) m over the pair's 32 edges (K = 32); first, so that m's split dies here
        wgrad_pair(accW, scW, gz3a, gz3b, mah, mal, mbh, mbl, img, e, g, lane, fmaxf(cma, cmb));
        STAMP(15);
        PAIR_FENCE();
        // z3 = Wc1 m + bc1: gm = Wc1^T gz3 + gM_r (M = sum_j m); gz2 = gm SiLU'(z2) -> pass B
        f4 gz2a[4], gz2b[4];
        load_ecl(gz2a, sGM + ga.rl * ROWP, g);
        load_ecl(gz2b, sGM + gb.rl * ROWP, g);
        if (!ga.rv) zero4(gz2a);
        if (!gb.rv) zero4(gz2b);
        mm64_cs2(gz2a, gz2b, hWc1T, gz3a, gz3b, lane, us_wc1t, cma, cmb);
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) { gz2a[mt] *= d2a[mt]; gz2b[mt] *= d2b[mt]; }
        STAMP(3);
        PAIR_FENCE();
        {   // the handoff blocks (rows past the range too: their slots lie inside the unit's block)
          float* da = p.stash + ga.su * HID;
          float* db = p.stash + gb.su * HID;
#pragma unroll
          for (int mt = 0; mt < 4; ++mt) {
            *reinterpret_cast<f4*>(da + mt * 256 + e * 16 + 4 * g) = gz2a[mt];
            *reinterpret_cast<f4*>(db + mt * 256 + e * 16 + 4 * g) = gz2b[mt];
          }
          if (g == 0) {
            p.stash_c[ga.su + e] = ca;
            p.stash_c[gb.su + e] = cb;
          }
        }
        STAMP(4);
        STAMP(15);
      }
    }
    if constexpr (PAIRS) {
      // the single-unit form after the pair loop: the units of pairs flagged in bigmask, then the odd
      // last unit
      const int nbig = 2 * __builtin_popcountll(bigmask);
      const int nrun = nbig + (u_first < U ? 1 : 0);
      for (int t = 0; t < nrun; ++t) {
        int uu = u_first;
        if (t < nbig) {
          unsigned long long mm = bigmask;
          for (int b = 0; b < (t >> 1); ++b) mm &= mm - 1;
          uu = 2 * (wave + NW * __builtin_ctzll(mm)) + (t & 1);
        }
        int tau_u, k_u;
        unit_tk(uu, tau_u, k_u);
        const LT lt_u = lane_tile(tau_u);
        prefetch(lt_u, k_u);
        float fe_in[NEP];
#pragma unroll
        for (int kk = 0; kk < NEP; ++kk) fe_in[kk] = efn[kk];
        f4 gz_in[4];
        float c_in = 0.f;
        if constexpr (PASS == 1) {
#pragma unroll
          for (int mt = 0; mt < 4; ++mt) gz_in[mt] = gzn[mt];
          c_in = cn;
        } else {
          zero4(gz_in);
        }
        unit_one(lt_u, k_u, fe_in, gz_in, c_in);
      }
    } else {
      // the current and the next unit as (tile geometry, sender offset), stepped by NW units
      int tau_n, k_n;
      unit_tk(u_first < U ? u_first : 0, tau_n, k_n);
      LT lt_n = lane_tile(tau_n);
      int k_c = k_n;
      LT lt_c = lt_n;
      if (u_first < U) prefetch(lt_n, k_n);
      for (int u = u_first; u < U; u += NW) {
        // the weight fragments are loop-invariant: without this barrier the compiler hoists all four
        // 64x64 matrices (256 VGPRs) out of the loop and spills
        asm volatile("" ::: "memory");
        float fe_in[NEP];
#pragma unroll
        for (int kk = 0; kk < NEP; ++kk) fe_in[kk] = efn[kk];
        f4 gz_in[4];
        float c_in = 0.f;
        if constexpr (PASS == 1) {
#pragma unroll
          for (int mt = 0; mt < 4; ++mt) gz_in[mt] = gzn[mt];
          c_in = cn;
        }
        if (u + NW < U) {
          step_tk(tau_n, k_n, NW);
          if (tau_n != lt_n.tau) lt_n = lane_tile(tau_n);
        }
        prefetch(lt_n, k_n);
        unit_one(lt_c, k_c, fe_in, gz_in, c_in);
        lt_c = lt_n;
        k_c = k_n;
      }
    }
    if (PASS == 1 && cur_tau >= 0) flush_ga(cur_tau);
    STAMP(PASS ? 7 : 15);
    __syncthreads();
    STAMP(PASS ? 10 : 14);
    if (PASS == 0) continue;
    // ---- C: write the chunk's sums (senders can be shared with the next chunk: atomics) ----
    // (the four wave-private tables added in wave order)
    for (int i = tid; i < ctc * 16 * HID; i += NW * 64) {
      const int rl = i / HID, ch = i - rl * HID;
      const int r = rbase + rl;
      const int o = rl * ROWP + ch;
      if (r < nend) p.GA[(size_t)r * HID + ch] = ((sGA[o] + sGA[rows * ROWP + o]) + sGA[2 * rows * ROWP + o]) +
                                                 sGA[3 * rows * ROWP + o];
    }
    for (int i = tid; i < (gtab ? 0 : S * HID); i += NW * 64) {
      const int sl = i / HID, ch = i - sl * HID;
      const int o = sl * ROWP + ch, st = p.s_max * ROWP;
      atomicAdd(p.GB + (size_t)(s0 + sl) * HID + ch, ((sGB[o] + sGB[st + o]) + sGB[2 * st + o]) + sGB[3 * st + o]);
    }
    for (int i = tid; i < (gtab ? 0 : S * 3); i += NW * 64) {
      const int sl = i / 3, d = i - 3 * sl;
      const int o = sl * 4 + d, st = p.s_max * 4;
      atomicAdd(p.GX + (size_t)(s0 + sl) * 4 + d, ((sGX[o] + sGX[st + o]) + sGX[2 * st + o]) + sGX[3 * st + o]);
    }
    __syncthreads();
    STAMP(11);
  }
  // ---- D: weight-gradient partials: each wave's to LDS, then one per block (waves added in order) ----
  __syncthreads();   // the last chunk's tables are dead: reuse the LDS
  float* wp = smem + wave * EW_STRIDE;
  auto put = [&](const f4 (&acc)[4][4], float sc, int wo) {
    const float inv_sc = 1.f / sc;   // exact (power of two)
    if constexpr (PAIRS) {
      // acc in image-column order on both axes (wgrad_pair / wgrad_h16<true>): un-permuted here; bias:
      // lane (e, g) holds channel 16 mt + 4 g + q summed over its edges; add the 16 edges
#pragma unroll
      for (int ot = 0; ot < 4; ++ot)
#pragma unroll
        for (int it = 0; it < 4; ++it)
#pragma unroll
          for (int q = 0; q < 4; ++q)
            wp[wo + chan_img(ot, 4 * g + q) * 65 + chan_img(it, e)] = acc[ot][it][q] * inv_sc;
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float b = edge_sum16(bsE[mt][q]);
          if (e == 0) wp[wo + (16 * mt + 4 * g + q) * 65 + 64] = b;
        }
    } else {
#pragma unroll
      for (int ot = 0; ot < 4; ++ot)
#pragma unroll
        for (int it = 0; it < 4; ++it)
#pragma unroll
          for (int q = 0; q < 4; ++q) wp[wo + (16 * ot + 4 * g + q) * 65 + 16 * it + e] = acc[ot][it][q] * inv_sc;
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const float bs = group_sum(sB[t]) * inv_sc;
        if (g == 0) wp[wo + (16 * t + e) * 65 + 64] = bs;
      }
    }
  };
  put(accW, scW, PASS == 0 ? EW_WC1 : EW_W2);
  if (PASS == 1) {
#pragma unroll
    for (int f = 0; f < NF; ++f)
#pragma unroll
      for (int ot = 0; ot < 4; ++ot)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float v = edge_sum16(accFe[f][ot][q]);
          if (e == 0) wp[EW_FEAT + (16 * ot + 4 * g + q) * (NF + 1) + f] = v;
        }
    if (e == 0)
#pragma unroll
      for (int ot = 0; ot < 4; ++ot)
#pragma unroll
        for (int q = 0; q < 4; ++q) wp[EW_FEAT + (16 * ot + 4 * g + q) * (NF + 1) + NF] = 0.f;
  }
  if (PASS == 0) {
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float wc2 = edge_sum16(sWC2[mt][q]);
        if (e == 0) wp[EW_WC2 + 16 * mt + 4 * g + q] = wc2;
      }
    const float gcs = edge_sum16(sGC);   // every lane group holds the same gc per edge: take group 0
    if (lane == 0) wp[EW_WC2 + 64] = gcs;
  }
  float* dst = p.wpart + (size_t)blockIdx.x * EW_STRIDE;
  block_partial(smem, dst, PASS == 0 ? EW_WC1 : EW_W2, PASS == 1 ? EW_WC1 : EW_WC2 + 65);
  if (PASS == 1) block_partial(smem, dst, EW_FEAT, EW_FEAT + 64 * (NF + 1));
  STAMP(12);
  STAMP_FLUSH
}

template <int NE, int PASS>
__global__ __launch_bounds__(256) void edge_bwd_kernel(EdgeBwdArgs p) {
  if (p.bb[BOFF_SCAL + SC_NORM] != 0.f) edge_bwd_body<NE, PASS, 1, 2>(p);        // wave-uniform
  else if (p.bb[BOFF_SCAL + SC_TANH] != 0.f) edge_bwd_body<NE, PASS, 2, 2>(p);
  else if (p.segno) {
    if constexpr (PASS == 1) {
      if (p.gtab) { edge_bwd_body<NE, PASS, 3, 1>(p); return; }
    }
    edge_bwd_body<NE, PASS, 3, 0>(p);
  } else {
    if constexpr (PASS == 1) {
      if (p.gtab) { edge_bwd_body<NE, PASS, 0, 1>(p); return; }
    }
    edge_bwd_body<NE, PASS, 0, 0>(p);
  }
}
// per-pass chunk size (tiles per LDS chunk) and dynamic LDS bytes
// (gtab_out: pass B takes the large-N form, EdgeBwdArgs::gtab, when its sender tables do not fit)
int edge_bwd_config(int pass, int n_graphs, int N, int G, int* ct_out, int* s_max_out, size_t* lds_out,
                    int* gtab_out = nullptr) {
  const int tiles_per = (((n_graphs + G - 1) / G) * N + 15) / 16;
  int ct = 8 < tiles_per ? 8 : tiles_per;
  while (ct > 1 && ct * (N - 1) > 512) --ct;   // pass A's per-wave pair mask: <= 64 pairs per wave and chunk
  static const int force_gtab = getenv_int("NONODE_GTAB");   // (A/B switch: the large-N form at any N)
  int s_max = 0, gtab = pass == 1 && force_gtab;
  while (ct > 1 && edge_bwd_lds_floats(pass, ct, N, &s_max, gtab) * 4 > 160 * 1024) --ct;
  size_t lds = edge_bwd_lds_floats(pass, ct, N, &s_max, gtab) * 4;
  if (lds > 160 * 1024 && pass == 1) {
    gtab = 1;
    lds = edge_bwd_lds_floats(pass, ct, N, &s_max, 1) * 4;
  }
  if (lds > 160 * 1024 || ct * (N - 1) > 512)
    return fail(NONODE_EUNSUPPORTED, "edge backward: N=%d too large (pass %d LDS tables %zu bytes > 160 KB)", N, pass, lds);
  const size_t red = (size_t)4 * EW_STRIDE * 4;   // the end-of-kernel partial combine
  lds = lds > red ? lds : red;
  *ct_out = ct; *s_max_out = s_max; *lds_out = lds;
  if (gtab_out) *gtab_out = gtab;
  return NONODE_OK;
}

// grid of the edge backward over n_graphs graphs (one workgroup per CU, at most EB_MAX_BLOCKS)
int edge_bwd_grid(int n_graphs) {
  int G = num_cus();
  G = G < EB_MAX_BLOCKS ? G : EB_MAX_BLOCKS;
  return n_graphs < G ? n_graphs : G;
}
// the entry points check that both passes' LDS tables fit before any launch, naming themselves
int edge_bwd_fits(const char* who, int n_graphs, int N) {
  int ct, s_max;
  size_t lds;
  for (int pass = 0; pass < 2; ++pass)
    if (edge_bwd_config(pass, n_graphs, N, edge_bwd_grid(n_graphs), &ct, &s_max, &lds))
      return fail(NONODE_EUNSUPPORTED, "%s: N=%d too large for the edge backward (pass %d LDS tables > 160 KB; "
                  "training supports N <= %d)", who, N, pass, EB_N_MAX);
  return NONODE_OK;
}

int launch_edge_bwd(int ne, EdgeBwdArgs a, int G, hipStream_t s) {
  static std::once_flag once[5];
  auto go = [&](void (*k0)(EdgeBwdArgs), void (*k1)(EdgeBwdArgs)) {
    std::call_once(once[ne], [&] {
      hipFuncSetAttribute((const void*)k0, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      hipFuncSetAttribute((const void*)k1, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    });
    size_t lds = 0;
    if (int rc = edge_bwd_config(0, a.n_graphs, a.N, G, &a.ct, &a.s_max, &lds)) return rc;
    {
      ProfScope prof(PROF_EDGE_BWD0, s);
      hipLaunchKernelGGL(k0, dim3(G), dim3(256), lds, s, a);
    }
    if (int rc = check_launch("edge_bwd_kernel<pass 0>")) return rc;
    if (int rc = edge_bwd_config(1, a.n_graphs, a.N, G, &a.ct, &a.s_max, &lds, &a.gtab)) return rc;
    {
      ProfScope prof(PROF_EDGE_BWD1, s);
      hipLaunchKernelGGL(k1, dim3(G), dim3(256), lds, s, a);
    }
    return check_launch("edge_bwd_kernel<pass 1>");
  };
  switch (ne) {
    case 0: return go(edge_bwd_kernel<0, 0>, edge_bwd_kernel<0, 1>);
    case 1: return go(edge_bwd_kernel<1, 0>, edge_bwd_kernel<1, 1>);
    case 2: return go(edge_bwd_kernel<2, 0>, edge_bwd_kernel<2, 1>);
    case 3: return go(edge_bwd_kernel<3, 0>, edge_bwd_kernel<3, 1>);
    case 4: return go(edge_bwd_kernel<4, 0>, edge_bwd_kernel<4, 1>);
  }
  return fail(NONODE_EUNSUPPORTED, "edge_bwd: n_edge_feat=%d", ne);
}

// backward mixing fragments: mode m < M, c = re|im: frag(mo, mt)[lane][q] = W[i][o][m][c] with
// i = 16 mo + (l & 15), o = 16 mt + 4 (l >> 4) + q  (A operand over o, unscaled)
// (run by the extra workgroups of tconvx_bwd_kernel: one element per thread)
__device__ __forceinline__ void tconv_pack_bwd(const float* w, int Mfull, int M, float* out, int d) {
  if (d >= M * 2 * 4096) return;
  const int mat = d >> 12, r = d & 4095;
  const int m = mat >> 1, c = mat & 1;
  const int q = r & 3, l = (r >> 2) & 63, rest = r >> 8, mt = rest & 3, mo = rest >> 2;
  const int i = 16 * mo + (l & 15), o = 16 * mt + 4 * (l >> 4) + q;
  out[d] = w[(((size_t)i * 64 + o) * Mfull + m) * 2 + c];
}

// the TimeConv_x weight gradient from tconvx_bwd_kernel's per-block sums [nb][io][MMAX_T][2]: workgroup d
// (one per output of g_tconvx [2][2][Mfull][2], modes >= M zero; the extra workgroups of
// tconv_wgrad_reduce) adds the nb partial rows' entry with 256 threads (strided sums, then a fixed-order
// tree in LDS: deterministic). (One 256-thread block for every output, three lanes per output, had made
// this a 21 us serial chain per C4 layer.)
__device__ __forceinline__ void tconvx_grad_finish(const float* part, int nb, int M, int Mfull, float* dst, int d) {
  constexpr int cnt = 2 * 2 * MMAX_T * 2;   // partial row length (72)
  __shared__ float red[256];
  const int io = d / (Mfull * 2), m = (d / 2) % Mfull, c = d & 1;
  float v = 0.f;
  if (m < M) {
    const int k = (io * MMAX_T + m) * 2 + c;
    for (int r = threadIdx.x; r < nb; r += 256) v += part[(size_t)r * cnt + k];
  }
  red[threadIdx.x] = v;
  __syncthreads();
  for (int h = 128; h > 0; h >>= 1) {
    if ((int)threadIdx.x < h) red[threadIdx.x] += red[threadIdx.x + h];
    __syncthreads();
  }
  if (threadIdx.x == 0) dst[d] = red[0];
}

// TimeConv_x: X0 = [x - lm, v] per spatial dim, 2 channels, no activation. Writes gx, gv.
// One thread per (column c, coordinate d); the block sums its threads' weight-gradient terms in a
// fixed order and writes one row of 2*2*MMAX_T*2 partials (tconvx_grad_finish adds the blocks' rows).
// TB: compile-time frame bound (10 for T <= 10, else TMAX): the per-frame arrays are registers indexed
// by unrolled loops, and every frame's loads are issued up front, unconditionally with the frame index
// clamped to T - 1 (round 5 looped over a runtime T: per-frame loads behind a loop the compiler could not
// unroll, one memory latency per frame)
constexpr int TX_THREADS = 128;
template <int MM, int TB>
__global__ __launch_bounds__(TX_THREADS) void tconvx_bwd_kernel(int BN, int T, int M, int Mfull, const float* x,
                                                                const float* v, const float* lm, const float* gxo,
                                                                const float* gvo, const float* w, float* gx,
                                                                float* gv, float* part, int frames, int nbx,
                                                                const float* tw, float* twb) {
  if ((int)blockIdx.x >= nbx) {   // extra workgroups: the TimeConv backward's mixing fragments
    tconv_pack_bwd(tw, Mfull, M, twb, (blockIdx.x - nbx) * TX_THREADS + threadIdx.x);
    return;
  }
  constexpr int CNT = 2 * 2 * MM * 2;   // this build's partials; the row written is [io][MMAX_T][2]
  // twiddles cos / sin(pi 2 m t / T) once per block in LDS (the same float values a per-thread double
  // cospi / sinpi gave; that software double trig per thread had made this kernel ~38 us at C4)
  __shared__ float sCs[MM * TMAX], sSn[MM * TMAX];
  __shared__ float red[TX_THREADS][CNT + 1];
  for (int i = threadIdx.x; i < M * T; i += blockDim.x) {
    const int m = i / T, t = i - m * T;
    const double ang = 2.0 * (double)m * (double)t / (double)T;
    sCs[m * TMAX + t] = (float)cospi(ang);
    sSn[m * TMAX + t] = (float)sinpi(ang);
  }
  __syncthreads();
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  const bool valid = idx < BN * 3;
  const int c = valid ? idx / 3 : 0, d = valid ? idx - 3 * (idx / 3) : 0;
  float pp[CNT];
#pragma unroll
  for (int k = 0; k < CNT; ++k) pp[k] = 0.f;
  if (valid) {
    float X[2][TB], G[2][TB], GO[2][TB];
#pragma unroll
    for (int t = 0; t < TB; ++t) {
      const size_t row = (size_t)(t < T ? t : T - 1) * BN + c;
      X[0][t] = x[row * 3 + d] - lm[(frames ? row : (size_t)c) * 3 + d];
      X[1][t] = v[row * 3 + d];
      GO[0][t] = G[0][t] = gxo[row * 3 + d];
      GO[1][t] = G[1][t] = gvo[row * 3 + d];
    }
    // the 2 x 2 complex weights of every mode, requested before the mode loop (m clamped to M - 1)
    float wre[2][2][MM], wim[2][2][MM];
#pragma unroll
    for (int m = 0; m < MM; ++m)
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int o = 0; o < 2; ++o) {
          const int mc = m < M ? m : M - 1;
          wre[i][o][m] = w[((i * 2 + o) * Mfull + mc) * 2 + 0];
          wim[i][o][m] = w[((i * 2 + o) * Mfull + mc) * 2 + 1];
        }
#pragma unroll
    for (int m = 0; m < MM; ++m) {
      if (m >= M) break;
      const float cm = ((m == 0 || 2 * m == T) ? 1.f : 2.f) / (float)T;
      float Xr[2] = {0.f, 0.f}, Xi[2] = {0.f, 0.f}, gYr[2] = {0.f, 0.f}, gYi[2] = {0.f, 0.f};
#pragma unroll
      for (int t = 0; t < TB; ++t) {
        if (t >= T) break;
        const float cs = sCs[m * TMAX + t], sn = sSn[m * TMAX + t];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          Xr[i] = fmaf(X[i][t], cs, Xr[i]); Xi[i] = fmaf(-X[i][t], sn, Xi[i]);
          gYr[i] = fmaf(cm * cs, GO[i][t], gYr[i]); gYi[i] = fmaf(-cm * sn, GO[i][t], gYi[i]);
        }
      }
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        float gxr = 0.f, gxi = 0.f;
#pragma unroll
        for (int o = 0; o < 2; ++o) {
          const float wr = wre[i][o][m], wi = wim[i][o][m];
          gxr += gYr[o] * wr + gYi[o] * wi;
          gxi += -gYr[o] * wi + gYi[o] * wr;
          pp[((i * 2 + o) * MM + m) * 2 + 0] = Xr[i] * gYr[o] + Xi[i] * gYi[o];
          pp[((i * 2 + o) * MM + m) * 2 + 1] = -Xi[i] * gYr[o] + Xr[i] * gYi[o];
        }
#pragma unroll
        for (int t = 0; t < TB; ++t) {
          if (t >= T) break;
          G[i][t] += gxr * sCs[m * TMAX + t] - gxi * sSn[m * TMAX + t];
        }
      }
    }
#pragma unroll
    for (int t = 0; t < TB; ++t) {
      if (t >= T) break;
      const size_t row = (size_t)t * BN + c;
      gx[row * 3 + d] = G[0][t];
      gv[row * 3 + d] = G[1][t];
    }
  }
#pragma unroll
  for (int k = 0; k < CNT; ++k) red[threadIdx.x][k] = pp[k];
  __syncthreads();
  // the block's 128 rows added in a fixed tree: every thread sums 16 rows of one column (one serial
  // 128-row sum per column had been a ~4 us chain per block), then 8 partials per column
  constexpr int RG = TX_THREADS / 16;   // row groups
  __shared__ float red2[RG][CNT];
  for (int q = threadIdx.x; q < RG * CNT; q += TX_THREADS) {
    const int k = q % CNT, rg = q / CNT;
    float acc = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc += red[rg * 16 + r][k];
    red2[rg][k] = acc;
  }
  __syncthreads();
  if (threadIdx.x < CNT) {
    float acc = 0.f;
#pragma unroll
    for (int rg = 0; rg < RG; ++rg) acc += red2[rg][threadIdx.x];
    const int io = threadIdx.x / (MM * 2), rest = threadIdx.x - io * (MM * 2);   // rest = 2 m + c
    part[(size_t)blockIdx.x * (2 * 2 * MMAX_T * 2) + io * (MMAX_T * 2) + rest] = acc;
  }
}

// ---- embedding Linear gradient (egno.py:63-76 reversed) ------------------------------------------
// dW[o][k] = sum over the rows r = t BN + c of gh0[r][o] in[r][k] and db[o] = sum_r gh0[r][o], where the
// embedding's input row is in[r] = [h_in[frames ? r : c], trig[(c % Bt) T + t]]: the raw time embedding
// of the row's sample and frame (layer_no.py:8-17), which temb_kernel writes into the saved state in the
// training forward (h0_kernel saves h_in). The input rows themselves are never materialised.
// A block takes eg_tpb (>= 1) consecutive 64-row tiles: gh0 rows and input rows (zero past column ld) staged in
// LDS; thread (o, kg) sums column o of the gradient against the 4-column input blocks kg, kg + 4, ...
// (LDS broadcasts), wave 0 the bias too, so no cross-wave sum is needed. One partial per block in
// gemm_reduce's layout: column block cb (inputs 64 cb ..) is [blocks][64][nc_cb + 1], block 0's column
// nc_0 = the bias; gemm_reduce_batch adds them in block order (deterministic).
constexpr int EG_TILE = 64, EG_MAX_BLOCKS = 1024;
// consecutive tiles per block: 1, or more once the rows need more than EG_MAX_BLOCKS blocks (C4: 2 tiles
// in 800 blocks measured 27.8 us against 31.1 us for 1 tile in 1600 blocks; SEGNO's 160 tiles: 1 tile,
// 7.0 against 11.3 us)
inline int eg_tpb(long long rows) {
  const long long ntile = (rows + EG_TILE - 1) / EG_TILE;
  const long long t = (ntile + EG_MAX_BLOCKS - 1) / EG_MAX_BLOCKS;
  return (int)(t > 1 ? t : 1);
}
inline int eg_blocks(long long rows) {
  const long long ntile = (rows + EG_TILE - 1) / EG_TILE, t = eg_tpb(rows);
  return (int)((ntile + t - 1) / t);
}
template <int NCMAX>   // in_node + time-embedding columns, padded to a multiple of 16: <= 48 or <= 144
__global__ __launch_bounds__(256) void emb_grad_kernel(int BN, int T, int Bt, int din, int ncol, int frames,
                                                       const float* __restrict__ gh0, const float* __restrict__ hin,
                                                       const float* __restrict__ trig, float* __restrict__ part,
                                                       int tpb) {
  __shared__ float sG[EG_TILE][65];
  __shared__ __attribute__((aligned(16))) float sA[EG_TILE][NCMAX];
  __shared__ int sRow[EG_TILE][2];   // per tile row: h_in row, time-embedding row (-1: past the rows)
  const int tid = threadIdx.x, o = tid & 63, kg = tid >> 6;
  const int ld = din + ncol;
  const int n = BN * T;   // (the host checks n < 2^31)
  constexpr int NB = NCMAX / 4, NBT = NB / 4;   // 4-column input blocks (NCMAX: a multiple of 16), per thread
  static_assert(NCMAX % 16 == 0, "4 column blocks per thread group");
  f4 acc[NBT];
#pragma unroll
  for (int j = 0; j < NBT; ++j) acc[j] = f4{0.f, 0.f, 0.f, 0.f};
  float bsum = 0.f;
  for (int it = 0; it < tpb; ++it) {
    const int r0 = (blockIdx.x * tpb + it) * EG_TILE;
    if (r0 >= n) break;   // (block-uniform)
    __syncthreads();      // the previous tile's sums have read the LDS rows
    if (tid < EG_TILE) {
      const int r = r0 + tid;
      const int t = r / BN, c = r - t * BN;
      sRow[tid][0] = r < n ? (frames ? r : c) : -1;
      sRow[tid][1] = (c % Bt) * T + t;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {   // gh0 rows: 64 x 16 float4
      const int i = tid + 256 * u, rr = i >> 4;
      const f4 g4 = r0 + rr < n ? reinterpret_cast<const f4*>(gh0 + (size_t)(r0 + rr) * 64)[i & 15]
                                : f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int q = 0; q < 4; ++q) sG[rr][4 * (i & 15) + q] = g4[q];
    }
    __syncthreads();
    // input rows: thread (rr = tid / 4, kq = tid % 4) stages columns kq, kq + 4, ... of tile row rr, every
    // address first (a valid one for padding and rows past the range), then all loads, then the stores
    {
      constexpr int KE = NCMAX / 4;
      const int rr = tid >> 2, kq = tid & 3;
      const int hr = sRow[rr][0], tr = sRow[rr][1];
      const float* hrow = hin + (size_t)(hr >= 0 ? hr : 0) * din;
      const float* trow = trig + (size_t)tr * ncol - din;   // column k >= din of the row is trow[k]
      float val[KE];
#pragma unroll
      for (int u = 0; u < KE; ++u) {
        const int k = kq + 4 * u;
        const bool live = hr >= 0 && k < ld;
        val[u] = live ? (k < din ? hrow[k] : trow[k]) : 0.f;
      }
#pragma unroll
      for (int u = 0; u < KE; ++u) sA[rr][kq + 4 * u] = val[u];
    }
    __syncthreads();
#pragma unroll 4
    for (int rr = 0; rr < EG_TILE; ++rr) {
      const float gv = sG[rr][o];
      bsum += gv;
#pragma unroll
      for (int j = 0; j < NBT; ++j) {
        const f4 a = *reinterpret_cast<const f4*>(&sA[rr][4 * (kg + 4 * j)]);
#pragma unroll
        for (int q = 0; q < 4; ++q) acc[j][q] = fmaf(gv, a[q], acc[j][q]);
      }
    }
  }
  const int nc0 = ld < 64 ? ld : 64;
  const size_t base1 = (size_t)gridDim.x * 64 * (nc0 + 1);
  auto out_at = [&](int k) -> float* {   // k == ld: the bias
    if (k == ld) return part + ((size_t)blockIdx.x * 64 + o) * (nc0 + 1) + nc0;
    if (k < 64) return part + ((size_t)blockIdx.x * 64 + o) * (nc0 + 1) + k;
    return part + base1 + ((size_t)blockIdx.x * 64 + o) * (ld - 64 + 1) + (k - 64);
  };
#pragma unroll
  for (int j = 0; j < NBT; ++j)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int k = 4 * (kg + 4 * j) + q;
      if (k < ld) *out_at(k) = acc[j][q];
    }
  if (kg == 0) *out_at(ld) = bsum;
}

// dst[i*ld + (col0 + j)*cs] (+)= scale * sum_b partial[b][i][j], bias[i] (+)= scale * sum_b
// partial[b][i][N]. 256 threads = 16 outputs x 16 strided partial sums, combined in a fixed order
// (deterministic).
// (columns j >= split go to col1 + (j - split) instead: the [s | ... | e] blocks of edge W1)
__device__ __forceinline__ void gemm_reduce_body(const float* partial, int nblk, int M, int N, float* dst, int ld,
                                                 int col0, int cs, float* bias, int accumulate, float scale,
                                                 int split, int col1, long long pstride, int bx) {
  __shared__ float red[16][17];
  const int NO = M * (N + 1);
  if (bx * 16 >= NO) return;   // whole block (a batch's grid covers its largest job)
  const int ol = threadIdx.x & 15, part = threadIdx.x >> 4;
  const int o = bx * 16 + ol;
  // eight independent partial sums per thread (a fixed tree: deterministic), so the loads of a
  // thread are in flight together
  float s8[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (o < NO) {
    int b = part;
    for (; b + 7 * 16 < nblk; b += 8 * 16)
#pragma unroll
      for (int u = 0; u < 8; ++u) s8[u] += partial[(size_t)(b + 16 * u) * pstride + o];
    for (int u = 0; b < nblk; b += 16, ++u) s8[u & 7] += partial[(size_t)b * pstride + o];
  }
  float s = ((s8[0] + s8[1]) + (s8[2] + s8[3])) + ((s8[4] + s8[5]) + (s8[6] + s8[7]));
  red[part][ol] = s;
  __syncthreads();
  if (part != 0 || o >= NO) return;
  s = 0.f;
  for (int q = 0; q < 16; ++q) s += red[q][ol];
  s *= scale;
  const int i = o / (N + 1), j = o - i * (N + 1);
  if (j < N) {
    const int col = j < split ? col0 + j : col1 + (j - split);
    if (dst) { float* p = dst + (size_t)i * ld + (size_t)col * cs; *p = accumulate ? *p + s : s; }
  } else if (bias) {
    bias[i] = accumulate ? bias[i] + s : s;
  }
}
__global__ __launch_bounds__(256) void gemm_reduce(const float* partial, int nblk, int M, int N, float* dst, int ld,
                                                   int col0, int cs, float* bias, int accumulate, float scale,
                                                   int split, int col1, long long pstride) {
  gemm_reduce_body(partial, nblk, M, N, dst, ld, col0, cs, bias, accumulate, scale, split, col1, pstride, blockIdx.x);
}
// a batch of reductions in one launch (blockIdx.y = job)
struct ReduceJob {
  const float* partial; int nblk, M, N; float* dst; int ld, col0, cs; float* bias; int accumulate; float scale;
  int split, col1; long long pstride;
};
constexpr int REDUCE_BATCH_MAX = 12;
struct ReduceBatchArgs { ReduceJob j[REDUCE_BATCH_MAX]; };
__global__ __launch_bounds__(256) void gemm_reduce_batch(ReduceBatchArgs a) {
  const ReduceJob& r = a.j[blockIdx.y];
  gemm_reduce_body(r.partial, r.nblk, r.M, r.N, r.dst, r.ld, r.col0, r.cs, r.bias, r.accumulate, r.scale, r.split,
                   r.col1, r.pstride, blockIdx.x);
}
// the batch's arguments and its grid width (blocks per job)
int reduce_batch_args(const ReduceJob* jobs, int count, ReduceBatchArgs* a, int* gx) {
  if (count > REDUCE_BATCH_MAX) return fail(NONODE_EINVAL, "reduce batch of %d", count);
  *a = ReduceBatchArgs{};
  *gx = 1;
  for (int i = 0; i < count; ++i) {
    a->j[i] = jobs[i];
    const int NO = jobs[i].M * (jobs[i].N + 1);
    *gx = (NO + 15) / 16 > *gx ? (NO + 15) / 16 : *gx;
  }
  return NONODE_OK;
}
int launch_reduce_batch(const ReduceJob* jobs, int count, hipStream_t s) {
  if (count <= 0) return NONODE_OK;
  ReduceBatchArgs a;
  int gx = 1;
  if (int rc = reduce_batch_args(jobs, count, &a, &gx)) return rc;
  hipLaunchKernelGGL(gemm_reduce_batch, dim3(gx, count), dim3(256), 0, s, a);
  return check_launch("gemm_reduce_batch");
}

// dst weights1 [i][o][Mfull][2] = sum over nblk partials, modes < M. 256 threads = 64 outputs x 4
// strided partial lanes, combined in a fixed order (deterministic). The same launch runs
// tconvx_grad_finish (the TimeConv_x weight gradient, xpart -> g_txw) and the EGNN layer's reductions
// (gemm_reduce_batch jobs, deferred to here) in its further workgroups.
struct TconvReduceArgs {
  const float* part; int nblk, M, Mfull; float* dst;     // TimeConv weight gradient (tconv_bwd partials)
  int nred;                                              // its workgroups
  const float* xpart; int nbx; float* g_txw; int nfin;   // TimeConv_x weight gradient: nfin workgroups
  ReduceBatchArgs rb; int rb_count, rb_gx;               // the EGNN layer's deferred reductions
};
__global__ __launch_bounds__(256) void tconv_wgrad_reduce(TconvReduceArgs a) {
  const int blk = blockIdx.x;
  if (blk >= a.nred + a.nfin) {   // a deferred gemm_reduce_batch job (rb_gx workgroups per job)
    const int b = blk - a.nred - a.nfin, jj = b / a.rb_gx;
    const ReduceJob& r = a.rb.j[jj];
    gemm_reduce_body(r.partial, r.nblk, r.M, r.N, r.dst, r.ld, r.col0, r.cs, r.bias, r.accumulate, r.scale, r.split,
                     r.col1, r.pstride, b - jj * a.rb_gx);
    return;
  }
  if (blk >= a.nred) {
    tconvx_grad_finish(a.xpart, a.nbx, a.M, a.Mfull, a.g_txw, blk - a.nred);
    return;
  }
  const float* part = a.part;
  const int nblk = a.nblk, M = a.M, Mfull = a.Mfull;
  float* dst = a.dst;
  // 16 outputs x 16 partial lanes per block, one float4 of 4 consecutive outputs per load (1 KB per
  // wave and partial row instead of 256 B; the scalar form ran at ~0.9 TB/s)
  __shared__ f4 red[16][17];
  const int per = M * 2 * 4096;
  const int ol = threadIdx.x & 15, pl = threadIdx.x >> 4;
  const int d4 = blk * 16 + ol;   // float4 index
  f4 s = f4{0.f, 0.f, 0.f, 0.f};
  if (4 * d4 < per)
    for (int b = pl; b < nblk; b += 16) s += reinterpret_cast<const f4*>(part + (size_t)b * per)[d4];
  red[pl][ol] = s;
  __syncthreads();
  if (threadIdx.x >= 64) return;
  const int oq = threadIdx.x >> 2, c4 = threadIdx.x & 3;   // output float4 oq, component c4
  const int d = 4 * (blk * 16 + oq) + c4;
  if (d >= per) return;
  float tot = 0.f;
  for (int q = 0; q < 16; ++q) tot += red[q][oq][c4];
  const int mc = d >> 12, r = d & 4095, m = mc >> 1, c = mc & 1, i = r >> 6, o = r & 63;
  dst[(((size_t)i * 64 + o) * Mfull + m) * 2 + c] = tot;
}


// ---- state layout of the training forward ---------------------------------------------------------
struct TrainState {
  unsigned long long* mask;   // L x T x ntiles x 16: TimeConv LeakyReLU decisions (TconvArgs::mask_out)
  float *hs, *xs, *vs;        // (L+1) x n x {64, 3, 3}: inputs of each layer's TimeConv (hs[0] = h0)
  float *he, *xe, *ve;        // L x n x {64, 3, 3}: TimeConv outputs = EGNN inputs
  float *Ms, *Fs;             // L x n x {64, 4}: message / force sums of each EGNN layer
  // embedding Linear inputs for its weight gradient (emb_grad_kernel): h_in rows (BN, or n with per-frame
  // inputs) x in_node, then the time-embedding table [Bt][T][temb] (temb_kernel's trig values); the
  // region is sized n x (in_node + temb), which holds both for any Bt dividing B N
  float *ein;
  size_t floats;
};
TrainState train_state(void* base, int B, int N, int T, int L, int in_node, int temb) {
  const size_t n = (size_t)B * N * T;
  TrainState st;
  float* p = (float*)base;
  auto take = [&](size_t cnt) { float* q = p; if (p) p += cnt; return q; };
  const size_t mask_words = (size_t)L * T * (((size_t)B * N + 15) / 16) * 16;
  st.mask = reinterpret_cast<unsigned long long*>(take(2 * mask_words));   // first: 8-byte aligned
  st.hs = take((L + 1) * n * 64); st.xs = take((L + 1) * n * 3); st.vs = take((L + 1) * n * 3);
  st.he = take(L * n * 64); st.xe = take(L * n * 3); st.ve = take(L * n * 3);
  st.Ms = take(L * n * 64); st.Fs = take(L * n * 4);
  st.ein = take(n * (in_node + temb));
  st.floats = (size_t)(2 * mask_words + (L + 1) * n * 70 + L * n * 70 + L * n * 68 + n * (in_node + temb));
  return st;
}

// backward workspace
struct BwdWs {
  float *gx[2], *gv[2], *gh[2];          // ping-pong grads of the current layer outputs (n rows)
  float *gF, *gM, *ghp, *GA, *GB, *GX, *gxe, *gve, *ghe;
  float *op_gt, *op_z, *op_gz, *p6;
  float *wpart;
  float *stash, *stash_c;                // edge backward pass A -> pass B ((N - 1) n rows)
  float *Pn, *Qn;                        // edge backward pass A -> pass B: node projections (n rows)
  float *twb, *tpart, *xpart;
  float *partial;
  size_t floats;
};
BwdWs bwd_ws(void* base, int B, int N, int T, int M) {
  const size_t BN = (size_t)B * N, n = BN * T;
  BwdWs w;
  float* p = (float*)base;
  size_t tot = 0;
  auto take = [&](size_t cnt) { float* q = p ? p + tot : nullptr; tot += (cnt + 63) & ~size_t(63); return q; };
  for (int i = 0; i < 2; ++i) { w.gx[i] = take(n * 3); w.gv[i] = take(n * 3); w.gh[i] = take(n * 64); }
  w.gF = take(n * 4); w.gM = take(n * 64); w.ghp = take(n * 64); w.GA = take(n * 64); w.GB = take(n * 64);
  w.GX = take(n * 4); w.gxe = take(n * 3); w.gve = take(n * 3); w.ghe = take(n * 64);
  w.op_gt = take(n * 64); w.op_z = take(n * 64); w.op_gz = take(n * 64);
  w.p6 = take((size_t)nonode_tu::NB_MAX_PARTS * 65);   // node_bwd's node_v output-row partials
  w.wpart = take((size_t)EB_MAX_BLOCKS * EW_STRIDE);
  const size_t npad = n + 16 * EB_MAX_BLOCKS;   // (N - 1) x (n + 16 G) handoff rows, G <= EB_MAX_BLOCKS
  w.stash = take(npad * (N - 1) * 64); w.stash_c = take(npad * (N - 1));
  w.Pn = take(n * 64); w.Qn = take(n * 64);
  w.twb = take((size_t)M * 2 * 4096);
  w.tpart = take((size_t)TB_MAX_BLOCKS * M * 2 * 4096);
  w.xpart = take((BN * 3 + TX_THREADS - 1) / TX_THREADS * (2 * 2 * MMAX_T * 2));   // one row per tconvx block
  // node_wgrad_kernel's partials (one [NW_JOBS][64][65] per block), or emb_grad_kernel's (one
  // [64][<= 137 + 2] per block: two column blocks)
  const size_t gparts = (size_t)eg_blocks((long long)n) * 64 * (8 + 2 * 64 + 2);
  const size_t nparts = (size_t)nonode_tu::NW_MAX_BLOCKS * nonode_tu::NW_JOBS * nonode_tu::NW_PART;
  w.partial = take(gparts > nparts ? gparts : nparts);
  w.floats = tot;
  return w;
}

}  // namespace

namespace {
// the validated PackArgs of one layer's backward blob (nonode_pack_layer_bwd's rules)
int pack_bwd_args(const nonode_layer_weights* w, int variant, int hidden, int n_edge_feat, float* bblob,
                  PackArgs* out) {
  if (!w || !bblob) return fail(NONODE_EINVAL, "pack_layer_bwd: null pointer");
  const int flags = variant & ~0xff;
  variant &= 0xff;
  if (flags & ~(NONODE_LAYER_NORM_RADIAL | NONODE_LAYER_TANH_COORD))
    return fail(NONODE_EINVAL, "pack_layer_bwd: unknown option bits 0x%x", flags);
  if (((flags & NONODE_LAYER_NORM_RADIAL) && variant != NONODE_VARIANT_EGNO) ||
      ((flags & NONODE_LAYER_TANH_COORD) && variant != NONODE_VARIANT_SEGNO))
    return fail(NONODE_EINVAL, "pack_layer_bwd: NORM_RADIAL is an EGNO option, TANH_COORD a SEGNO one");
  if (hidden != HID || n_edge_feat < 0 || n_edge_feat > 4)
    return fail(NONODE_EUNSUPPORTED, "pack_layer_bwd: hidden=%d n_edge_feat=%d", hidden, n_edge_feat);
  const bool egno = variant == NONODE_VARIANT_EGNO;
  if (!egno && variant != NONODE_VARIANT_SEGNO) return fail(NONODE_EINVAL, "pack_layer_bwd: variant %d", variant);
  if (!w->edge_w1 || !w->edge_b1 || !w->edge_w2 || !w->edge_b2 || !w->coord_w1 || !w->coord_b1 ||
      !w->coord_w2 || !w->coord_b2 || !w->node_w1 || !w->node_b1 || !w->node_w2 || !w->node_b2)
    return fail(NONODE_EINVAL, "pack_layer_bwd: missing weight pointer");
  if (egno && (!w->vel_w1 || !w->vel_b1 || !w->vel_w2 || !w->vel_b2))
    return fail(NONODE_EINVAL, "pack_layer_bwd: EGNO needs node_v_net weights");
  PackArgs& a = *out;
  a.ld1 = 2 * HID + 1 + n_edge_feat;
  if (egno) { a.colS = 0; a.colA = 1; a.colB = 1 + HID; }       // [s, h_i, h_j, e]  basic.py:152-154
  else { a.colA = 0; a.colB = HID; a.colS = 2 * HID; }          // [h_i, h_j, s, e]  gcl.py:78
  a.w1 = w->edge_w1; a.b1 = w->edge_b1; a.w2 = w->edge_w2; a.b2 = w->edge_b2;
  a.cw1 = w->coord_w1; a.cb1 = w->coord_b1; a.cw2 = w->coord_w2; a.cb2 = w->coord_b2;
  a.vw1 = egno ? w->vel_w1 : nullptr; a.vb1 = egno ? w->vel_b1 : nullptr;
  a.vw2 = egno ? w->vel_w2 : nullptr; a.vb2 = egno ? w->vel_b2 : nullptr;
  a.nw1 = w->node_w1; a.nb1 = w->node_b1; a.nw2 = w->node_w2; a.nb2 = w->node_b2;
  a.ne = n_edge_feat;
  a.flags = flags;
  a.blob = bblob;
  return NONODE_OK;
}
}  // namespace

extern "C" {

size_t nonode_bwd_blob_floats(void) { return BBLOB_FLOATS; }

int nonode_pack_layer_bwd(const nonode_layer_weights* w, int variant, int hidden, int n_edge_feat, float* bblob,
                          void* stream) {
  return nonode_pack_layers_bwd(&w, 1, variant, hidden, n_edge_feat, &bblob, stream);
}
int nonode_pack_layers_bwd(const nonode_layer_weights* const* w, int n_layers, int variant, int hidden,
                           int n_edge_feat, float* const* bblobs, void* stream) {
  if (!w || !bblobs || n_layers < 0) return fail(NONODE_EINVAL, "pack_layer_bwd: null pointer");
  // every layer is validated before the first launch: a bad entry leaves every blob untouched
  std::vector<PackArgs> args(n_layers);
  for (int l = 0; l < n_layers; ++l)
    if (int rc = pack_bwd_args(w[l], variant, hidden, n_edge_feat, bblobs[l], &args[l])) return rc;
  for (int l0 = 0; l0 < n_layers; l0 += PACK_MAX) {
    const int cnt = n_layers - l0 < PACK_MAX ? n_layers - l0 : PACK_MAX;
    PackBatch pb{};
    for (int k = 0; k < cnt; ++k) pb.a[k] = args[l0 + k];
    hipLaunchKernelGGL(pack_bwd_kernel, dim3(32, 31, cnt), dim3(256), 0, (hipStream_t)stream, pb);
    if (int rc = check_launch("pack_bwd_kernel")) return rc;
  }
  return NONODE_OK;
}

size_t nonode_egno_train_state_bytes(int B, int N, int T, int n_layers, int in_node, int time_emb_dim) {
  return train_state(nullptr, B, N, T, n_layers, in_node, time_emb_dim).floats * sizeof(float);
}

}  // extern "C"

namespace {
// frames = 1: per-frame inputs (num_inputs > 1) and, with t_in, the input-time embedding columns
int egno_forward_train_impl(int frames, int B, int N, int T, int n_layers, int in_node, int n_edge_feat,
                              int time_emb_dim, int modes, int Bt, const float* x, const float* h, const float* v,
                              const float* loc_mean, const float* edge_fea, const float* t_in, const float* t_out,
                              const float* emb_w, const float* emb_b, const float* const* blobs,
                              const float* const* tconv_blobs, const float* const* tconvx_w, float* x_out,
                              float* v_out, float* h_out, void* state, size_t state_bytes, void* workspace,
                              size_t workspace_bytes, void* stream) {
  if (B <= 0 || N < 2 || T <= 0 || T > TMAX || n_layers < 1 || in_node < 0 || in_node > 8 || modes < 1 ||
      modes > MMAX_T || time_emb_dim < 4 || time_emb_dim > 64 || (time_emb_dim & 1) || Bt <= 0 || (B * N) % Bt)
    return fail(NONODE_EUNSUPPORTED, "egno_forward_train: B=%d N=%d T=%d modes=%d (training: modes <= %d)", B, N, T,
                modes, MMAX_T);
  const bool tc = tconv_blobs != nullptr;   // false: use_time_conv=False (both TimeConv arrays null)
  if (!x || !h || !v || (tc && !loc_mean) || !t_out || !emb_w || !emb_b || !blobs || tc != (tconvx_w != nullptr) ||
      !x_out || !v_out || !h_out || !state || !workspace)
    return fail(NONODE_EINVAL, "egno_forward_train: null pointer");
  const int emb_cols = (t_in ? 2 : 1) * time_emb_dim;   // time-embedding columns of the embedding Linear
  if (state_bytes < nonode_egno_train_state_bytes(B, N, T, n_layers, in_node, emb_cols))
    return fail(NONODE_EINVAL, "egno_forward_train: state too small");
  if (workspace_bytes < nonode_egno_workspace_bytes(B, N, T, Bt))
    return fail(NONODE_EINVAL, "egno_forward_train: workspace too small");
  hipStream_t s = (hipStream_t)stream;
  const int BN = B * N;
  const size_t n = (size_t)BN * T;
  const int L = n_layers;
  TrainState st = train_state(state, B, N, T, L, in_node, emb_cols);
  float* etab = (float*)workspace + n * 64 + n * 3;
  const int emb_ld = in_node + emb_cols;
  {
    // temb_kernel also saves the raw time-embedding table and h0_kernel the h_in rows: the inputs of the
    // embedding's weight gradient (emb_grad_kernel)
    hipLaunchKernelGGL(temb_kernel, dim3((Bt * T + TEMB_ROWS - 1) / TEMB_ROWS), dim3(256), 0, s, Bt, T, in_node, time_emb_dim, t_out,
                       emb_w, emb_ld, emb_b, etab, t_in, st.ein + n * in_node);
    if (int rc = check_launch("temb_kernel")) return rc;
    hipLaunchKernelGGL(h0_kernel, dim3((BN * 64 + 255) / 256), dim3(256), 0, s, BN, T, in_node, Bt, h, emb_w, emb_ld,
                       etab, x, v, st.hs, st.xs, st.vs, frames, st.ein);
    if (int rc = check_launch("h0_kernel")) return rc;
  }
  // EGNN_Layer leaves v unchanged (basic.py:186): layer l's input v is TimeConv_x's output ve[l - 1]
  // (vs[0] without time convolutions); the last layer writes x_out, h_out directly
  for (int l = 0; l < L; ++l) {
    TconvArgs a{};
    a.BN = BN; a.T = T; a.M = effective_modes(T, modes); a.Mfull = modes;
    a.h = st.hs + l * n * 64; a.x = st.xs + l * n * 3; a.lm = loc_mean;
    a.v = (l > 0 && tc) ? st.ve + (l - 1) * n * 3 : st.vs;
    const float *hin, *xin, *vin;
    if (tc) {
      a.wp = tconv_blobs[l]; a.wx = tconvx_w[l]; a.frames = frames;
      a.h_out = st.he + l * n * 64; a.x_out = st.xe + l * n * 3; a.v_out = st.ve + l * n * 3;
      a.mask_out = st.mask + (size_t)l * T * ((BN + 15) / 16) * 16;
      if (int rc = launch_tconv(false, a, s)) return rc;
      hin = a.h_out; xin = a.x_out; vin = a.v_out;
    } else {   // the layer reads its saved inputs directly (the backward does the same)
      hin = a.h; xin = a.x; vin = a.v;
    }
    const bool last = l == L - 1;
    if (int rc = launch_layer<EGNO>(T * B, N, n_edge_feat, frames ? T * B : B, hin, xin, vin, edge_fea, blobs[l], 0.f,
                                    1.f, 0, last ? h_out : st.hs + (l + 1) * n * 64,
                                    last ? x_out : st.xs + (l + 1) * n * 3, nullptr, s, 1, nullptr,
                                    st.Ms + l * n * 64, st.Fs + l * n * 4, tc ? BN : 0))   // XCD order as the TimeConv's
      return rc;
  }
  hipMemcpyAsync(v_out, tc ? st.ve + (L - 1) * n * 3 : st.vs, n * 3 * sizeof(float), hipMemcpyDeviceToDevice, s);
  return check_launch("egno_forward_train copies");
}
}  // namespace

extern "C" {

int nonode_egno_forward_train(int B, int N, int T, int n_layers, int in_node, int n_edge_feat, int time_emb_dim,
                              int modes, int Bt, const float* x, const float* h, const float* v,
                              const float* loc_mean, const float* edge_fea, const float* t_out,
                              const float* emb_w, const float* emb_b, const float* const* blobs,
                              const float* const* tconv_blobs, const float* const* tconvx_w, float* x_out,
                              float* v_out, float* h_out, void* state, size_t state_bytes, void* workspace,
                              size_t workspace_bytes, void* stream) {
  return egno_forward_train_impl(0, B, N, T, n_layers, in_node, n_edge_feat, time_emb_dim, modes, Bt, x, h, v,
                                 loc_mean, edge_fea, nullptr, t_out, emb_w, emb_b, blobs, tconv_blobs, tconvx_w,
                                 x_out, v_out, h_out, state, state_bytes, workspace, workspace_bytes, stream);
}

int nonode_egno_forward_train_frames(int B, int N, int T, int n_layers, int in_node, int n_edge_feat,
                                     int time_emb_dim, int modes, int Bt, const float* x, const float* h,
                                     const float* v, const float* loc_mean, const float* edge_fea,
                                     const float* t_in, const float* t_out, const float* emb_w, const float* emb_b,
                                     const float* const* blobs, const float* const* tconv_blobs,
                                     const float* const* tconvx_w, float* x_out, float* v_out, float* h_out,
                                     void* state, size_t state_bytes, void* workspace, size_t workspace_bytes,
                                     void* stream) {
  return egno_forward_train_impl(1, B, N, T, n_layers, in_node, n_edge_feat, time_emb_dim, modes, Bt, x, h, v,
                                 loc_mean, edge_fea, t_in, t_out, emb_w, emb_b, blobs, tconv_blobs, tconvx_w,
                                 x_out, v_out, h_out, state, state_bytes, workspace, workspace_bytes, stream);
}

size_t nonode_egno_backward_workspace_bytes(int B, int N, int T, int modes) {
  return bwd_ws(nullptr, B, N, T, effective_modes(T, modes)).floats * sizeof(float);
}

}  // extern "C"

namespace {
// Reverse of ONE EGNN_Layer (basic.py:167-186) over n rows = n_graphs x N given its inputs (he, xe,
// ve), the forward's message / force sums (Ms, Fs) and the gradients of its outputs (gx, gv, gh):
// writes every parameter gradient of the layer (*lg) and the gradients of its inputs (g_*in).
// Shared by nonode_egno_backward (per layer) and nonode_egnn_layer_bwd.
struct LayerRev {
  int n, N, n_graphs, ef_mod, ne;
  const float *he, *xe, *ve, *Ms, *Fs, *edge_fea, *bb;
  const float *gx, *gv, *gh;
  const nonode_layer_grads* lg;
  float *g_xin, *g_vin, *g_hin;
};
// defer (non-null): the layer's reductions are returned in *defer (count in defer->n) for a later
// launch (tconv_reverse runs them beside its own) instead of launched here
struct DeferredReduce { ReduceJob j[REDUCE_BATCH_MAX]; int n = 0; };
int egnn_layer_reverse(const LayerRev& r, const BwdWs& w, hipStream_t s, DeferredReduce* defer = nullptr) {
  const size_t n = (size_t)r.n;
  const int N = r.N, ne = r.ne, ld1 = 2 * HID + 1 + ne;
  const nonode_layer_grads& lg = *r.lg;
  NodeBwdArgs na;
  na.n = r.n; na.N = N; na.h = r.he; na.v = r.ve; na.M = r.Ms; na.F = r.Fs;
  na.gxo = r.gx; na.gvo = r.gv; na.gho = r.gh; na.bb = r.bb;
  na.gv = r.g_vin; na.gF = w.gF; na.gM = w.gM; na.ghp = w.ghp;
  na.op_gt = w.op_gt; na.op_z = w.op_z; na.op_gz = w.op_gz; na.p6 = w.p6;
  const int ntile = (int)((n + 15) / 16);
  na.GB = w.GB; na.GX = w.GX;
  int n6 = 0;   // node_bwd's node_v output-row partial rows
  if (int rc = launch_node_bwd(na, ntile, s, &n6)) return rc;
  ReduceJob rjobs[REDUCE_BATCH_MAX];
  int nred = 0;
  {
    const int G = edge_bwd_grid(r.n_graphs);
    EdgeBwdArgs ea;
    ea.n_graphs = r.n_graphs; ea.N = N; ea.ne = ne; ea.ef_mod = r.ef_mod; ea.ct = 0; ea.s_max = 0; ea.gtab = 0;
    ea.segno = 0;
    ea.h = r.he; ea.x = r.xe; ea.ef = ne ? r.edge_fea : r.bb; ea.bb = r.bb; ea.gF = w.gF; ea.gM = w.gM;
    ea.GA = w.GA; ea.GB = w.GB; ea.GX = w.GX; ea.wpart = w.wpart;
    ea.stash = w.stash; ea.stash_c = w.stash_c; ea.Pn = w.Pn; ea.Qn = w.Qn;
    if (int rc = launch_edge_bwd(ne, ea, G, s)) return rc;
    // edge-level weight gradients: fixed-order sums of the G block partials (launched with the
    // node-level GEMMs' reductions below)
    const int nparts = G;   // one partial per block
    const int nf = 1 + ne;
    auto red = [&](int off, int M_, int N_, float* dst, int ld, float* bias, int split, int col1) {
      rjobs[nred++] = ReduceJob{w.wpart + off, nparts, M_, N_, dst, ld, 0, 1, bias, 0, 1.f, split, col1,
                                (long long)EW_STRIDE};
    };
    red(EW_W2, 64, 64, lg.edge_w2, 64, lg.edge_b2, 1 << 30, 0);
    red(EW_WC1, 64, 64, lg.coord_w1, 64, lg.coord_b1, 1 << 30, 0);
    red(EW_WC2, 1, 64, lg.coord_w2, 64, lg.coord_b2, 1 << 30, 0);
    // edge Linear 1 scalar columns [s | e] (EGNO order [s, h_i, h_j, e], basic.py:152-154, 170)
    red(EW_FEAT, 64, nf, lg.edge_w1, ld1, nullptr, 1, 2 * HID + 1);
  }
  const nonode_tu::NodePostArgs pa{r.n, w.ghp, w.GA, w.GB, r.gx, w.GX, r.bb, r.g_hin, r.g_xin};
  // ---- node-level weight gradients of this layer: one node_wgrad_kernel launch (NodeWgradArgs),
  // its and the edge-level reductions in another ----
  // edge Linear 1 h_i / h_j blocks; its bias gradient sum_e gz1 = sum_i GA_i comes with the h_i block
  {
    nonode_tu::NodeWgradArgs wa{};
    wa.n = (long long)n;
    wa.h = r.he; wa.M = r.Ms; wa.z = w.op_z;
    wa.GA = w.GA; wa.GB = w.GB; wa.gt = w.op_gt; wa.gz = w.op_gz; wa.gh = r.gh;
    wa.partial = w.partial;
    wa.post = pa;
    int nblk = 0;
    if (int rc = nonode_tu::launch_node_wgrad(wa, &nblk, s)) return rc;
    struct { float* dst; int ld, col0; float* bias; } d[nonode_tu::NW_JOBS + 1] = {
        {lg.edge_w1, ld1, 1, lg.edge_b1}, {lg.edge_w1, ld1, 1 + HID, nullptr}, {lg.vel_w1, 64, 0, lg.vel_b1},
        {lg.node_w1, 128, 0, lg.node_b1}, {lg.node_w1, 128, HID, nullptr},   {lg.node_w2, 64, 0, lg.node_b2},
        {lg.vel_w2, 64, 0, lg.vel_b2}};
    constexpr long long pstride = (long long)nonode_tu::NW_JOBS * nonode_tu::NW_PART;
    for (int j = 0; j < nonode_tu::NW_JOBS; ++j)
      rjobs[nred++] = ReduceJob{w.partial + (size_t)j * nonode_tu::NW_PART, nblk, 64, 64, d[j].dst, d[j].ld,
                                d[j].col0, 1, d[j].bias, 0, 1.f, 1 << 30, 0, pstride};
    // the node_v output row (d[6]) from node_bwd's per-workgroup partials
    rjobs[nred++] = ReduceJob{w.p6, n6, 1, 64, d[6].dst, d[6].ld, d[6].col0, 1, d[6].bias, 0, 1.f, 1 << 30, 0, 65};
    if (defer) {
      for (int i = 0; i < nred; ++i) defer->j[i] = rjobs[i];
      defer->n = nred;
      return NONODE_OK;
    }
    return launch_reduce_batch(rjobs, nred, s);
  }
}

// Reverse of TimeConv + TimeConv_x of one EGNO layer (layer_no.py:80-178, egno.py:99-108): given the
// layer's TimeConv inputs (h [T][BN][64], x, v) and the gradients of its outputs (gh, gx, gv), writes
// the input gradients (g_hin, g_xin, g_vin) and the raw weight gradients (g_tw [64][64][modes][2],
// g_txw [2][2][modes][2]). mask: the forward's LeakyReLU decisions (TconvArgs::mask_out).
struct TconvRev {
  int BN, T, M, modes, frames;
  const float *hs, *xs, *vs, *lm, *tw, *txw;
  const unsigned long long* mask;
  const float *gh, *gx, *gv;
  float *g_hin, *g_xin, *g_vin, *g_tw, *g_txw;
};
int tconv_reverse(const TconvRev& r, const BwdWs& w, hipStream_t s, const DeferredReduce* defer = nullptr) {
  const int BN = r.BN, T = r.T, M = r.M, modes = r.modes;
  // g_txw [2][2][Mfull][2]: one partial row per tconvx block, added in block order (modes >= M zero)
  const int nbx = (BN * 3 + TX_THREADS - 1) / TX_THREADS;
  // mode-bound builds: 2 (C4), 4, 9 (registers of the per-thread partials)
  auto txk = T <= 10 ? (M <= 2 ? tconvx_bwd_kernel<2, 10> : (M <= 4 ? tconvx_bwd_kernel<4, 10> : tconvx_bwd_kernel<MMAX_T, 10>))
                    : (M <= 2 ? tconvx_bwd_kernel<2, TMAX> : (M <= 4 ? tconvx_bwd_kernel<4, TMAX> : tconvx_bwd_kernel<MMAX_T, TMAX>));
  // (+ the workgroups that pack the TimeConv backward's fragments, tconv_pack_bwd)
  const int npack = (M * 2 * 4096 + TX_THREADS - 1) / TX_THREADS;
  hipLaunchKernelGGL(txk, dim3(nbx + npack), dim3(TX_THREADS), 0, s, BN, T, M, modes, r.xs, r.vs,
                     r.lm, r.gx, r.gv, r.txw, r.g_xin, r.g_vin, w.xpart, r.frames, nbx, r.tw, w.twb);
  if (int rc = check_launch("tconvx_bwd_kernel")) return rc;
  TconvBwdArgs ta;
  ta.BN = BN; ta.T = T; ta.M = M; ta.ntiles = (BN + 15) / 16;
  ta.h = r.hs; ta.gout = r.gh; ta.wb = w.twb; ta.gh = r.g_hin; ta.wpart = w.tpart;
  ta.mask = r.mask;
  int TG = num_cus();
  TG = TG < TB_MAX_BLOCKS ? TG : TB_MAX_BLOCKS;
  const int tgw = (ta.ntiles + tb_groups(M) - 1) / tb_groups(M);   // workgroups: tb_groups(M) tiles each per trip
  TG = tgw < TG ? tgw : TG;
  if (int rc = launch_tconv_bwd(M, ta, TG, s)) return rc;
  if (modes > M) hipMemsetAsync(r.g_tw, 0, (size_t)64 * 64 * modes * 2 * sizeof(float), s);   // bins >= M
  const int nred = (M * 2 * 4096 / 4 + 15) / 16;   // (+ one tconvx_grad_finish workgroup per g_txw entry)
  TconvReduceArgs ra;
  ra.part = w.tpart; ra.nblk = TG; ra.M = M; ra.Mfull = modes; ra.dst = r.g_tw; ra.nred = nred;
  ra.xpart = w.xpart; ra.nbx = nbx; ra.g_txw = r.g_txw; ra.nfin = 4 * modes * 2;
  ra.rb_count = defer ? defer->n : 0;
  ra.rb_gx = 1;
  if (ra.rb_count > 0) {
    if (int rc = reduce_batch_args(defer->j, defer->n, &ra.rb, &ra.rb_gx)) return rc;
  } else {
    ra.rb = ReduceBatchArgs{};
  }
  hipLaunchKernelGGL(tconv_wgrad_reduce, dim3(nred + ra.nfin + ra.rb_count * ra.rb_gx), dim3(256), 0, s, ra);
  return check_launch("tconv_wgrad_reduce");
}

// frames = 1: per-frame loc_mean / edge_fea (num_inputs > 1); emb_cols: time-embedding columns of
// the embedding Linear (time_emb_dim, or 2 time_emb_dim with the input-time embedding)
int egno_backward_impl(int frames, int emb_cols, int B, int N, int T, int n_layers, int in_node, int n_edge_feat,
                         int time_emb_dim, int modes, int Bt, const float* loc_mean, const float* edge_fea,
                         const float* const* bblobs, const float* const* tconv_w, const float* const* tconvx_w,
                         const void* state, const float* g_x, const float* g_v, const float* g_h,
                         const nonode_layer_grads* layer_grads, float* const* g_tconv, float* const* g_tconvx,
                         float* g_emb_w, float* g_emb_b, void* workspace, size_t workspace_bytes, void* stream) {
  if (B <= 0 || N < 2 || T <= 0 || T > TMAX || n_layers < 1 || modes < 1 || modes > MMAX_T || Bt <= 0 ||
      n_edge_feat < 0 || n_edge_feat > 4)
    return fail(NONODE_EUNSUPPORTED, "egno_backward: B=%d N=%d T=%d", B, N, T);
  const bool tc = tconv_w != nullptr;   // false: use_time_conv=False (every TimeConv array null)
  if ((tc && (!loc_mean || !tconvx_w || !g_tconv || !g_tconvx)) ||
      (!tc && (tconvx_w || g_tconv || g_tconvx)) || !bblobs || !state || !g_x || !layer_grads ||
      !g_emb_w || !g_emb_b || !workspace || (n_edge_feat > 0 && !edge_fea))
    return fail(NONODE_EINVAL, "egno_backward: null pointer");
  if (int rc = edge_bwd_fits("egno_backward", B * T, N)) return rc;
  const int M = effective_modes(T, modes);
  if (workspace_bytes < nonode_egno_backward_workspace_bytes(B, N, T, modes))
    return fail(NONODE_EINVAL, "egno_backward: workspace too small");
  hipStream_t s = (hipStream_t)stream;
  const int BN = B * N, L = n_layers, ne = n_edge_feat;
  const size_t n = (size_t)BN * T;
  const long long E = (long long)n * (N - 1);
  TrainState st = train_state(const_cast<void*>(state), B, N, T, L, in_node, emb_cols);
  BwdWs w = bwd_ws(workspace, B, N, T, M);
  // grads of the final outputs
  // (read in place: the reverse pass only reads the output gradients of a layer)
  const float *gx = g_x, *gv = g_v, *gh = g_h;
  if (!g_v) { hipMemsetAsync(w.gv[0], 0, n * 3 * sizeof(float), s); gv = w.gv[0]; }
  if (!g_h) { hipMemsetAsync(w.gh[0], 0, n * 64 * sizeof(float), s); gh = w.gh[0]; }
  int cur = 0;
  for (int l = L - 1; l >= 0; --l) {
    const float* he = (tc ? st.he : st.hs) + l * n * 64;
    const float* xe = (tc ? st.xe : st.xs) + l * n * 3;
    const float* ve = tc ? st.ve + l * n * 3 : st.vs;   // v is unchanged by every layer
    // ---- EGNN_Layer reverse ----
    LayerRev lr;
    lr.n = (int)n; lr.N = N; lr.n_graphs = T * B; lr.ef_mod = frames ? T * B : B; lr.ne = ne;
    lr.he = he; lr.xe = xe; lr.ve = ve; lr.Ms = st.Ms + l * n * 64; lr.Fs = st.Fs + l * n * 4;
    lr.edge_fea = edge_fea; lr.bb = bblobs[l];
    lr.gx = gx; lr.gv = gv; lr.gh = gh; lr.lg = &layer_grads[l];
    lr.g_xin = w.gxe; lr.g_vin = w.gve; lr.g_hin = w.ghe;
    DeferredReduce dr;   // with TimeConv, the layer's reductions run in tconv_reverse's last launch
    if (int rc = egnn_layer_reverse(lr, w, s, tc ? &dr : nullptr)) return rc;
    const int nxt = cur ^ 1;
    if (!tc) {   // no TimeConv: the layer-input gradients are the next (earlier) layer's output gradients
      hipMemcpyAsync(w.gx[nxt], w.gxe, n * 3 * sizeof(float), hipMemcpyDeviceToDevice, s);
      hipMemcpyAsync(w.gv[nxt], w.gve, n * 3 * sizeof(float), hipMemcpyDeviceToDevice, s);
      hipMemcpyAsync(w.gh[nxt], w.ghe, n * 64 * sizeof(float), hipMemcpyDeviceToDevice, s);
      if (int rc = check_launch("egno_backward copies")) return rc;
      cur = nxt;
      gx = w.gx[cur]; gv = w.gv[cur]; gh = w.gh[cur];
      continue;
    }
    // ---- TimeConv_x / TimeConv reverse: x, v, h of the layer's TimeConv input ----
    TconvRev tr;
    tr.BN = BN; tr.T = T; tr.M = M; tr.modes = modes; tr.frames = frames;
    tr.hs = st.hs + l * n * 64; tr.xs = st.xs + l * n * 3; tr.vs = l > 0 ? st.ve + (l - 1) * n * 3 : st.vs;
    tr.lm = loc_mean; tr.tw = tconv_w[l]; tr.txw = tconvx_w[l];
    tr.mask = st.mask + (size_t)l * T * ((BN + 15) / 16) * 16;
    tr.gh = w.ghe; tr.gx = w.gxe; tr.gv = w.gve;
    tr.g_hin = w.gh[nxt]; tr.g_xin = w.gx[nxt]; tr.g_vin = w.gv[nxt]; tr.g_tw = g_tconv[l]; tr.g_txw = g_tconvx[l];
    if (int rc = tconv_reverse(tr, w, s, &dr)) return rc;
    cur = nxt;
    gx = w.gx[cur]; gv = w.gv[cur]; gh = w.gh[cur];
  }
  // ---- embedding Linear (egno.py:63-76): dW = sum_rows gh0 (x) [h_in, temb], db = sum gh0 ----
  {
    const int emb_ld = in_node + emb_cols;
    if (n >= (size_t)1 << 31) return fail(NONODE_EUNSUPPORTED, "egno_backward: %zu embedding rows", n);
    const int nblk = eg_blocks((long long)n), tpb = eg_tpb((long long)n);
    const float* hin_s = st.ein;
    const float* trig_s = st.ein + n * in_node;
    if (emb_ld <= 48)
      hipLaunchKernelGGL(emb_grad_kernel<48>, dim3(nblk), dim3(256), 0, s, BN, T, Bt, in_node, emb_cols, frames, gh,
                         hin_s, trig_s, w.partial, tpb);
    else
      hipLaunchKernelGGL(emb_grad_kernel<144>, dim3(nblk), dim3(256), 0, s, BN, T, Bt, in_node, emb_cols, frames, gh,
                         hin_s, trig_s, w.partial, tpb);
    if (int rc = check_launch("emb_grad_kernel")) return rc;
    const int nc0 = emb_ld < 64 ? emb_ld : 64;
    ReduceJob jobs[2];
    jobs[0] = ReduceJob{w.partial, nblk, 64, nc0, g_emb_w, emb_ld, 0, 1, g_emb_b, 0, 1.f, 1 << 30, 0,
                        (long long)64 * (nc0 + 1)};
    int nj = 1;
    if (emb_ld > 64)
      jobs[nj++] = ReduceJob{w.partial + (size_t)nblk * 64 * (nc0 + 1), nblk, 64, emb_ld - 64, g_emb_w, emb_ld, 64, 1,
                             nullptr, 0, 1.f, 1 << 30, 0, (long long)64 * (emb_ld - 64 + 1)};
    if (int rc = launch_reduce_batch(jobs, nj, s)) return rc;
  }
  return NONODE_OK;
}
}  // namespace

extern "C" {

int nonode_egno_backward(int B, int N, int T, int n_layers, int in_node, int n_edge_feat, int time_emb_dim,
                         int modes, int Bt, const float* loc_mean, const float* edge_fea,
                         const float* const* bblobs, const float* const* tconv_w, const float* const* tconvx_w,
                         const void* state, const float* g_x, const float* g_v, const float* g_h,
                         const nonode_layer_grads* layer_grads, float* const* g_tconv, float* const* g_tconvx,
                         float* g_emb_w, float* g_emb_b, void* workspace, size_t workspace_bytes, void* stream) {
  return egno_backward_impl(0, time_emb_dim, B, N, T, n_layers, in_node, n_edge_feat, time_emb_dim, modes, Bt,
                            loc_mean, edge_fea, bblobs, tconv_w, tconvx_w, state, g_x, g_v, g_h, layer_grads, g_tconv,
                            g_tconvx, g_emb_w, g_emb_b, workspace, workspace_bytes, stream);
}

int nonode_egno_backward_frames(int B, int N, int T, int n_layers, int in_node, int n_edge_feat, int time_emb_dim,
                                int with_t_in, int modes, int Bt, const float* loc_mean, const float* edge_fea,
                                const float* const* bblobs, const float* const* tconv_w,
                                const float* const* tconvx_w, const void* state, const float* g_x, const float* g_v,
                                const float* g_h, const nonode_layer_grads* layer_grads, float* const* g_tconv,
                                float* const* g_tconvx, float* g_emb_w, float* g_emb_b, void* workspace,
                                size_t workspace_bytes, void* stream) {
  return egno_backward_impl(1, (with_t_in ? 2 : 1) * time_emb_dim, B, N, T, n_layers, in_node, n_edge_feat,
                            time_emb_dim, modes, Bt, loc_mean, edge_fea, bblobs, tconv_w, tconvx_w, state, g_x, g_v,
                            g_h, layer_grads, g_tconv, g_tconvx, g_emb_w, g_emb_b, workspace, workspace_bytes, stream);
}

}  // extern "C"

// ================================================================================================
// SEGNO training: forward_step (model.py:95-102) = T applications of SEGNO_GCL (gcl.py:111-119) with
// shared weights and dt = 1/T, run as T single-substep launches that save every substep's inputs and
// message / force sums; the reverse pass walks the substeps backwards on the EGNO backward kernels
// (edge_bwd_kernel with the per-edge clamp of gcl.py:99-100, node_wgrad_kernel) and adds
// every substep's weight gradients into the same outputs. Replaces loss.backward() of
// train_nbody.py:168-179 through forward_step.
namespace {

struct SegnoNodeBwdArgs {
  int n, N, recurrent;
  float dt, cw;
  const float* h; const float* M;                       // substep inputs h, saved message sums
  const float* gxo; const float* gvo; const float* gho;  // grads of the substep outputs
  const float* bb;
  float* gv; float* gF; float* gM; float* ghp;           // outputs
  float* op_z; float* op_gz;                             // GEMM operands (node MLP weight gradients)
  float* GB; float* GX;                                  // the edge backward's sender sums: zeroed here
  int nmain;                                             // workgroups of the node reverse; further ones:
  ReduceBatchArgs rb; int rb_count, rb_gx;               // the previous substep's deferred reductions
};

// reverse of  v' = v + cw mean_j clamp(r_ij c_ij) dt ;  x' = x + v' dt   (gcl.py:255-257, 242)
//             h' = [h +] WN2 SiLU(WN1 [h, M] + bn1) + bn2                 (gcl.py:85-95)
// gF is the gradient of the per-receiver sum of the clamped edge translations (the per-edge clamp
// mask is applied by edge_bwd_kernel, which recomputes r c)
__global__ __launch_bounds__(256) void segno_node_bwd_kernel(SegnoNodeBwdArgs p) {
  if ((int)blockIdx.x >= p.nmain) {   // a deferred gemm_reduce_batch job (rb_gx workgroups per job)
    const int b = (int)blockIdx.x - p.nmain, jj = b / p.rb_gx;
    const ReduceJob& r = p.rb.j[jj];
    gemm_reduce_body(r.partial, r.nblk, r.M, r.N, r.dst, r.ld, r.col0, r.cs, r.bias, r.accumulate, r.scale, r.split,
                     r.col1, r.pstride, b - jj * p.rb_gx);
    return;
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, e = lane & 15, g = lane >> 4;
  const int r0 = (blockIdx.x * 4 + wave) * 16;
  if (r0 >= p.n) return;
  const int r = min(r0 + e, p.n - 1);
  const bool valid = r0 + e < p.n;
  const float* bb = p.bb;
  f4 hr[4], Mr[4], in8[8];
  load_ecl(hr, p.h + (size_t)r * HID, g);
  load_ecl(Mr, p.M + (size_t)r * HID, g);
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) { in8[mt] = hr[mt]; in8[4 + mt] = Mr[mt]; }
  f4 zp[4], z[4];
  load_vp(zp, bb + BOFF_VEC + BV_BN1 * 64, g);
  mfma_dense<8>(zp, bb + BOFF_WN1, in8, lane);
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) z[mt] = zp[mt];
  silu_true(z);
  f4 gho[4], gz[4], gh[4], gM[4];
  load_ecl(gho, p.gho + (size_t)r * HID, g);
  zero4(gz);
  mfma_dense<4>(gz, bb + BOFF_WN2T, gho, lane);
  mul_dsilu(gz, zp);
  if (p.recurrent) {
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) gh[mt] = gho[mt];
  } else {
    zero4(gh);
  }
  mfma_dense<4>(gh, bb + BOFF_WN1TH, gz, lane);
  zero4(gM);
  mfma_dense<4>(gM, bb + BOFF_WN1TM, gz, lane);
  if (valid) {
    const size_t o = (size_t)r * HID;
    store_ecl(p.ghp + o, gh, g);
    store_ecl(p.gM + o, gM, g);
    store_ecl(p.op_z + o, z, g);
    store_ecl(p.op_gz + o, gz, g);
    const f4 z4[4] = {};
    store_ecl(p.GB + o, z4, g);
    if (g == 0) {
      *reinterpret_cast<f4*>(p.GX + (size_t)r * 4) = z4[0];
      const float f = p.dt * p.cw / (float)(p.N - 1);
      float gvt[3];
#pragma unroll
      for (int d = 0; d < 3; ++d) {
        gvt[d] = p.gvo[(size_t)r * 3 + d] + p.gxo[(size_t)r * 3 + d] * p.dt;
        p.gv[(size_t)r * 3 + d] = gvt[d];
      }
      *reinterpret_cast<f4*>(p.gF + (size_t)r * 4) = f4{gvt[0] * f, gvt[1] * f, gvt[2] * f, 0.f};
    }
  }
}

struct SegnoState {
  float *hs, *xs, *vs;   // (T + 1) x n x {64, 3, 3}: substep inputs (index T: the result)
  float* Ms;             // T x n x 64: message sums of each substep (the reverse pass recomputes the
                         // per-edge forces and clamp masks itself, so no force sums are kept)
  size_t floats;
};
SegnoState segno_state(void* base, int B, int N, int T) {
  const size_t n = (size_t)B * N;
  SegnoState st;
  float* p = (float*)base;
  auto take = [&](size_t cnt) { float* q = p; if (p) p += cnt; return q; };
  st.hs = take((T + 1) * n * 64); st.xs = take((T + 1) * n * 3); st.vs = take((T + 1) * n * 3);
  st.Ms = take(T * n * 64);
  st.floats = (size_t)(T + 1) * n * 70 + (size_t)T * n * 64;
  return st;
}

}  // namespace

extern "C" {

size_t nonode_segno_train_state_bytes(int B, int N, int T) {
  return segno_state(nullptr, B, N, T < 0 ? 0 : T).floats * sizeof(float);
}

int nonode_segno_forward_train(int B, int N, int T, int n_edge_feat, const float* h, const float* x,
                               const float* v, const float* edge_attr, const float* blob, float coords_weight,
                               int recurrent, float* x_out, float* v_out, float* h_out, void* state,
                               size_t state_bytes, void* stream) {
  if (B <= 0 || N < 2 || T < 0 || n_edge_feat < 0 || n_edge_feat > 4)
    return fail(NONODE_EUNSUPPORTED, "segno_forward_train: B=%d N=%d T=%d ne=%d", B, N, T, n_edge_feat);
  if (!h || !x || !v || !blob || !x_out || !v_out || !h_out || !state || (n_edge_feat > 0 && !edge_attr))
    return fail(NONODE_EINVAL, "segno_forward_train: null pointer");
  if (state_bytes < nonode_segno_train_state_bytes(B, N, T))
    return fail(NONODE_EINVAL, "segno_forward_train: state too small");
  hipStream_t s = (hipStream_t)stream;
  const size_t n = (size_t)B * N;
  SegnoState st = segno_state(state, B, N, T);
  hipMemcpyAsync(st.hs, h, n * 64 * sizeof(float), hipMemcpyDeviceToDevice, s);
  hipMemcpyAsync(st.xs, x, n * 3 * sizeof(float), hipMemcpyDeviceToDevice, s);
  hipMemcpyAsync(st.vs, v, n * 3 * sizeof(float), hipMemcpyDeviceToDevice, s);
  if (T == 0) {
    hipMemcpyAsync(h_out, h, n * 64 * sizeof(float), hipMemcpyDeviceToDevice, s);
    hipMemcpyAsync(x_out, x, n * 3 * sizeof(float), hipMemcpyDeviceToDevice, s);
    hipMemcpyAsync(v_out, v, n * 3 * sizeof(float), hipMemcpyDeviceToDevice, s);
    return check_launch("segno_forward_train");
  }
  // all T substeps in one launch of the inference layer kernel (fused substeps where a workgroup owns
  // one whole-graph chunk), saving every substep's outputs and message sums (LayerArgs::sv_h)
  float* const sv[3] = {st.hs, st.xs, st.vs};
  if (int rc = launch_layer<SEGNO>(B, N, n_edge_feat, B, h, x, v, edge_attr, blob, 1.0f / (float)T, coords_weight,
                                   recurrent, h_out, x_out, v_out, s, T, nullptr, st.Ms, nullptr, 0, sv))
    return rc;
  return check_launch("segno_forward_train");
}

size_t nonode_segno_backward_workspace_bytes(int B, int N) {
  return bwd_ws(nullptr, B, N, 1, 1).floats * sizeof(float);
}

int nonode_segno_backward(int B, int N, int T, int n_edge_feat, float coords_weight, int recurrent,
                          const float* edge_attr, const float* bblob, const void* state, const float* g_x,
                          const float* g_v, const float* g_h, const nonode_layer_grads* grads, float* g_h_in,
                          float* g_x_in, float* g_v_in, void* workspace, size_t workspace_bytes, void* stream) {
  if (B <= 0 || N < 2 || T < 0 || n_edge_feat < 0 || n_edge_feat > 4)
    return fail(NONODE_EUNSUPPORTED, "segno_backward: B=%d N=%d T=%d ne=%d", B, N, T, n_edge_feat);
  if (!bblob || !state || !grads || !workspace || (n_edge_feat > 0 && !edge_attr))
    return fail(NONODE_EINVAL, "segno_backward: null pointer");
  const nonode_layer_grads& lg = *grads;
  if (!lg.edge_w1 || !lg.edge_b1 || !lg.edge_w2 || !lg.edge_b2 || !lg.coord_w1 || !lg.coord_b1 || !lg.coord_w2 ||
      !lg.coord_b2 || !lg.node_w1 || !lg.node_b1 || !lg.node_w2 || !lg.node_b2)
    return fail(NONODE_EINVAL, "segno_backward: missing gradient pointer");
  if (workspace_bytes < nonode_segno_backward_workspace_bytes(B, N))
    return fail(NONODE_EINVAL, "segno_backward: workspace too small");
  if (int rc = edge_bwd_fits("segno_backward", B, N)) return rc;
  hipStream_t s = (hipStream_t)stream;
  const int ne = n_edge_feat, ld1 = 2 * HID + 1 + ne;
  const size_t n = (size_t)B * N;
  const SegnoState st = segno_state(const_cast<void*>(state), B, N, T);
  BwdWs w = bwd_ws(workspace, B, N, 1, 1);
  // the output gradients are read in place (every kernel only reads them); null ones are zeros
  const float *gx = g_x, *gv = g_v, *gh = g_h;
  if (!g_x) { hipMemsetAsync(w.gx[0], 0, n * 3 * sizeof(float), s); gx = w.gx[0]; }
  if (!g_v) { hipMemsetAsync(w.gv[0], 0, n * 3 * sizeof(float), s); gv = w.gv[0]; }
  if (!g_h) { hipMemsetAsync(w.gh[0], 0, n * 64 * sizeof(float), s); gh = w.gh[0]; }
  if (T == 0) {   // no substep: every weight gradient is zero, the input gradients pass through
    hipMemsetAsync(lg.edge_w1, 0, (size_t)64 * ld1 * sizeof(float), s);
    for (float* q : {lg.edge_w2, lg.coord_w1, lg.node_w2}) hipMemsetAsync(q, 0, 64 * 64 * sizeof(float), s);
    hipMemsetAsync(lg.node_w1, 0, 64 * 128 * sizeof(float), s);
    for (float* q : {lg.edge_b1, lg.edge_b2, lg.coord_b1, lg.coord_w2, lg.node_b1, lg.node_b2})
      hipMemsetAsync(q, 0, 64 * sizeof(float), s);
    hipMemsetAsync(lg.coord_b2, 0, sizeof(float), s);
  }
  const int ntile = (int)((n + 15) / 16);
  int cur = 0;
  // each substep's weight-gradient reductions run in extra workgroups of the next (earlier) substep's
  // segno_node_bwd_kernel launch (they touch none of its buffers; the partials they read are only
  // overwritten by the edge backward after it), the last substep's in their own launch
  ReduceJob prev[REDUCE_BATCH_MAX];
  int nprev = 0;
  for (int t = T - 1; t >= 0; --t) {
    const int acc = t < T - 1;   // substeps share the weights: add into the gradients after the first
    const float* hs = st.hs + t * n * 64;
    const float* Ms = st.Ms + t * n * 64;
    const int nxt = cur ^ 1;
    SegnoNodeBwdArgs na;
    na.n = (int)n; na.N = N; na.recurrent = recurrent; na.dt = 1.0f / (float)T; na.cw = coords_weight;
    na.h = hs; na.M = Ms; na.gxo = gx; na.gvo = gv; na.gho = gh; na.bb = bblob;
    // the first substep's input gradients go straight to the caller's outputs (when they alias no input)
    auto out_to = [&](float* dst, const float* in0, const float* in1, float* ws) {
      return (t == 0 && dst && dst != in0 && dst != in1) ? dst : ws;
    };
    float* gv_o = out_to(g_v_in, g_v, g_x, w.gv[nxt]);
    float* gh_o = out_to(g_h_in, g_h, nullptr, w.gh[nxt]);
    float* gx_o = out_to(g_x_in, g_x, g_v, w.gx[nxt]);
    na.gv = gv_o; na.gF = w.gF; na.gM = w.gM; na.ghp = w.ghp; na.op_z = w.op_z; na.op_gz = w.op_gz;
    na.GB = w.GB; na.GX = w.GX;
    na.nmain = (ntile + 3) / 4;
    na.rb_count = nprev; na.rb_gx = 1;
    if (nprev)
      if (int rc = reduce_batch_args(prev, nprev, &na.rb, &na.rb_gx)) return rc;
    hipLaunchKernelGGL(segno_node_bwd_kernel, dim3(na.nmain + nprev * na.rb_gx), dim3(256), 0, s, na);
    if (int rc = check_launch("segno_node_bwd_kernel")) return rc;
    ReduceJob rj[REDUCE_BATCH_MAX];   // the substep's edge- and node-level reductions: one launch
    int nrj = 0;
    {
      const int G = edge_bwd_grid(B);
      EdgeBwdArgs ea;
      ea.segno = 1;
      ea.n_graphs = B; ea.N = N; ea.ne = ne; ea.ef_mod = B; ea.ct = 0; ea.s_max = 0; ea.gtab = 0;
      ea.h = hs; ea.x = st.xs + t * n * 3; ea.ef = ne ? edge_attr : bblob; ea.bb = bblob; ea.gF = w.gF;
      ea.gM = w.gM; ea.GA = w.GA; ea.GB = w.GB; ea.GX = w.GX; ea.wpart = w.wpart;
      ea.stash = w.stash; ea.stash_c = w.stash_c; ea.Pn = w.Pn; ea.Qn = w.Qn;
      if (int rc = launch_edge_bwd(ne, ea, G, s)) return rc;
      auto red = [&](int off, int M_, int N_, float* dst, int ld, float* bias, int col0) {
        rj[nrj++] = ReduceJob{w.wpart + off, G, M_, N_, dst, ld, col0, 1, bias, acc, 1.f, 1 << 30, 0,
                              (long long)EW_STRIDE};
      };
      red(EW_W2, 64, 64, lg.edge_w2, 64, lg.edge_b2, 0);
      red(EW_WC1, 64, 64, lg.coord_w1, 64, lg.coord_b1, 0);
      red(EW_WC2, 1, 64, lg.coord_w2, 64, lg.coord_b2, 0);
      // edge Linear 1 scalar columns [s | e] (SEGNO order [h_i, h_j, s, e], gcl.py:78)
      red(EW_FEAT, 64, 1 + ne, lg.edge_w1, ld1, nullptr, 2 * HID);
    }
    const nonode_tu::NodePostArgs pa{(int)n, w.ghp, w.GA, w.GB, gx, w.GX, bblob, gh_o, gx_o};
    // node-level weight gradients of this substep (edge Linear 1 h_i / h_j blocks, node MLP): one
    // node_wgrad_kernel launch (jobs 0, 1, 3, 4, 5; no node_v MLP) and one reduction launch
    {
      nonode_tu::NodeWgradArgs wa{};
      wa.n = (long long)n;
      wa.h = hs; wa.M = Ms; wa.z = w.op_z;
      wa.GA = w.GA; wa.GB = w.GB; wa.gt = nullptr; wa.gz = w.op_gz; wa.gh = gh;
      wa.partial = w.partial;
      wa.post = pa;
      int nblk = 0;
      if (int rc = nonode_tu::launch_node_wgrad(wa, &nblk, s)) return rc;
      struct { int job; float* dst; int ld, col0; float* bias; } d[5] = {
          {0, lg.edge_w1, ld1, 0, lg.edge_b1}, {1, lg.edge_w1, ld1, HID, nullptr}, {3, lg.node_w1, 128, 0, lg.node_b1},
          {4, lg.node_w1, 128, HID, nullptr}, {5, lg.node_w2, 64, 0, lg.node_b2}};
      for (int j = 0; j < 5; ++j)
        rj[nrj++] = ReduceJob{w.partial + (size_t)d[j].job * nonode_tu::NW_PART, nblk, 64, 64, d[j].dst, d[j].ld,
                              d[j].col0, 1, d[j].bias, acc, 1.f, 1 << 30, 0,
                              (long long)nonode_tu::NW_JOBS * nonode_tu::NW_PART};
      for (int k = 0; k < nrj; ++k) prev[k] = rj[k];
      nprev = nrj;
    }
    cur = nxt;
    gx = gx_o; gv = gv_o; gh = gh_o;
  }
  if (int rc = launch_reduce_batch(prev, nprev, s)) return rc;
  if (g_h_in && g_h_in != gh) hipMemcpyAsync(g_h_in, gh, n * 64 * sizeof(float), hipMemcpyDeviceToDevice, s);
  if (g_x_in && g_x_in != gx) hipMemcpyAsync(g_x_in, gx, n * 3 * sizeof(float), hipMemcpyDeviceToDevice, s);
  if (g_v_in && g_v_in != gv) hipMemcpyAsync(g_v_in, gv, n * 3 * sizeof(float), hipMemcpyDeviceToDevice, s);
  return check_launch("segno_backward");
}

// ---- embedding Linear (SEGNO model.py:73: h = embedding(his)) as a forward / backward pair, so that a
// training caller keeps it off the autograd tape (its broadcast torch ops and their reverse were ~0.1 ms of
// the C3 training step)
int nonode_embedding_forward(int n_rows, int in_features, const float* in, const float* weight, const float* bias,
                             float* out, void* stream) {
  if (n_rows <= 0 || in_features < 1 || in_features > 40 || (size_t)n_rows * 64 >= ((size_t)1 << 31))
    return fail(NONODE_EUNSUPPORTED, "embedding_forward: rows=%d in_features=%d", n_rows, in_features);
  if (!in || !weight || !bias || !out) return fail(NONODE_EINVAL, "embedding_forward: null pointer");
  hipLaunchKernelGGL(embed_kernel, dim3((unsigned)(((size_t)n_rows * 64 + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, n_rows, in_features, in, weight, bias, out);
  return check_launch("embedding_forward");
}

size_t nonode_embedding_backward_workspace_bytes(int n_rows, int in_features) {
  if (n_rows <= 0 || in_features < 1) return 0;
  return (size_t)eg_blocks(n_rows) * 64 * (in_features + 1) * sizeof(float);
}

// grad_weight[o][k] = sum_n grad_out[n][o] in[n][k], grad_bias[o] = sum_n grad_out[n][o] (written, not
// accumulated): emb_grad_kernel with no time-embedding columns, then the block partials in block order
int nonode_embedding_backward(int n_rows, int in_features, const float* in, const float* grad_out,
                              float* grad_weight, float* grad_bias, void* workspace, size_t workspace_bytes,
                              void* stream) {
  if (n_rows <= 0 || in_features < 1 || in_features > 40)
    return fail(NONODE_EUNSUPPORTED, "embedding_backward: rows=%d in_features=%d", n_rows, in_features);
  if (!in || !grad_out || !grad_weight || !grad_bias || !workspace)
    return fail(NONODE_EINVAL, "embedding_backward: null pointer");
  if (workspace_bytes < nonode_embedding_backward_workspace_bytes(n_rows, in_features))
    return fail(NONODE_EINVAL, "embedding_backward: workspace too small");
  hipStream_t s = (hipStream_t)stream;
  const int nblk = eg_blocks(n_rows);
  float* part = (float*)workspace;
  hipLaunchKernelGGL(emb_grad_kernel<48>, dim3(nblk), dim3(256), 0, s, n_rows, 1, 1, in_features, 0, 0, grad_out, in,
                     in, part, eg_tpb(n_rows));   // (no time-embedding columns: trig is never read)
  if (int rc = check_launch("emb_grad_kernel")) return rc;
  const ReduceJob job{part, nblk, 64, in_features, grad_weight, in_features, 0, 1, grad_bias, 0, 1.f, 1 << 30, 0,
                      (long long)64 * (in_features + 1)};
  return launch_reduce_batch(&job, 1, s);
}

}  // extern "C"

// ---- layer-granular reverse entry points (egno_layer_bwd, spectral_tconv_bwd) ----
extern "C" {

size_t nonode_egnn_layer_bwd_workspace_bytes(int n_graphs, int N) {
  if (n_graphs <= 0 || N < 2) return 0;
  const size_t n = (size_t)n_graphs * N;
  return (bwd_ws(nullptr, n_graphs, N, 1, 1).floats + n * (64 + 4 + 64 + 4)) * sizeof(float);
}

int nonode_egnn_layer_bwd(int variant, int n_graphs, int N, int n_edge_feat, int ef_mod, const float* h,
                          const float* x, const float* v, const float* edge_fea, const float* blob,
                          const float* bblob, const float* g_x, const float* g_v, const float* g_h,
                          const nonode_layer_grads* grads, float* g_h_in, float* g_x_in, float* g_v_in,
                          void* workspace, size_t workspace_bytes, void* stream) {
  if ((variant & 0xff) != NONODE_VARIANT_EGNO)
    return fail(NONODE_EUNSUPPORTED, "egnn_layer_bwd: EGNO layers only (SEGNO: nonode_segno_backward)");
  if (n_graphs <= 0 || N < 2 || n_edge_feat < 0 || n_edge_feat > 4 || ef_mod <= 0 || n_graphs % ef_mod)
    return fail(NONODE_EUNSUPPORTED, "egnn_layer_bwd: n_graphs=%d N=%d ne=%d ef_mod=%d", n_graphs, N, n_edge_feat,
                ef_mod);
  if (!h || !x || !v || !blob || !bblob || !g_x || !grads || !g_h_in || !g_x_in || !g_v_in || !workspace ||
      (n_edge_feat > 0 && !edge_fea))
    return fail(NONODE_EINVAL, "egnn_layer_bwd: null pointer");
  if (workspace_bytes < nonode_egnn_layer_bwd_workspace_bytes(n_graphs, N))
    return fail(NONODE_EINVAL, "egnn_layer_bwd: workspace too small");
  if (int rc = edge_bwd_fits("egnn_layer_bwd", n_graphs, N)) return rc;
  hipStream_t s = (hipStream_t)stream;
  const size_t n = (size_t)n_graphs * N;
  BwdWs w = bwd_ws(workspace, n_graphs, N, 1, 1);
  float* Ms = (float*)workspace + w.floats;   // the forward's message / force sums (recomputed here)
  float* Fs = Ms + n * 64;
  float* ht = Fs + n * 4;                     // the forward's outputs (not needed, written by the recompute)
  float* xt = ht + n * 64;
  if (int rc = launch_layer<EGNO>(n_graphs, N, n_edge_feat, ef_mod, h, x, v, edge_fea, blob, 0.f, 1.f, 0, ht, xt,
                                  nullptr, s, 1, nullptr, Ms, Fs))
    return rc;
  const float *gv = g_v, *gh = g_h;
  if (!g_v) { hipMemsetAsync(w.gv[0], 0, n * 3 * sizeof(float), s); gv = w.gv[0]; }
  if (!g_h) { hipMemsetAsync(w.gh[0], 0, n * 64 * sizeof(float), s); gh = w.gh[0]; }
  LayerRev lr;
  lr.n = (int)n; lr.N = N; lr.n_graphs = n_graphs; lr.ef_mod = ef_mod; lr.ne = n_edge_feat;
  lr.he = h; lr.xe = x; lr.ve = v; lr.Ms = Ms; lr.Fs = Fs; lr.edge_fea = edge_fea; lr.bb = bblob;
  lr.gx = g_x; lr.gv = gv; lr.gh = gh; lr.lg = grads;
  lr.g_xin = g_x_in; lr.g_vin = g_v_in; lr.g_hin = g_h_in;
  return egnn_layer_reverse(lr, w, s);
}

size_t nonode_egno_tconv_bwd_workspace_bytes(int BN, int T, int modes) {
  if (BN <= 0 || T <= 0 || T > TMAX || modes < 1 || modes > MMAX_T) return 0;
  const size_t n = (size_t)BN * T;
  const size_t mask_floats = 2 * (size_t)T * ((BN + 15) / 16) * 16;
  return (mask_floats + bwd_ws(nullptr, BN, 1, T, effective_modes(T, modes)).floats + n * 70) * sizeof(float);
}

int nonode_egno_tconv_bwd(int BN, int T, int modes, const float* h, const float* x, const float* v,
                          const float* loc_mean, const float* tconv_blob, const float* tconv_w,
                          const float* tconvx_w, const float* g_h, const float* g_x, const float* g_v,
                          float* g_h_in, float* g_x_in, float* g_v_in, float* g_tconv_w, float* g_tconvx_w,
                          void* workspace, size_t workspace_bytes, void* stream) {
  if (BN <= 0 || T <= 0 || T > TMAX || modes < 1 || modes > MMAX_T)
    return fail(NONODE_EUNSUPPORTED, "egno_tconv_bwd: BN=%d T=%d modes=%d (training: modes <= %d)", BN, T, modes,
                MMAX_T);
  if (!h || !x || !v || !loc_mean || !tconv_blob || !tconv_w || !tconvx_w || !g_h_in || !g_x_in || !g_v_in ||
      !g_tconv_w || !g_tconvx_w || !workspace)
    return fail(NONODE_EINVAL, "egno_tconv_bwd: null pointer");
  if (workspace_bytes < nonode_egno_tconv_bwd_workspace_bytes(BN, T, modes))
    return fail(NONODE_EINVAL, "egno_tconv_bwd: workspace too small");
  hipStream_t s = (hipStream_t)stream;
  const int M = effective_modes(T, modes);
  const size_t n = (size_t)BN * T;
  const size_t mask_floats = 2 * (size_t)T * ((BN + 15) / 16) * 16;
  auto* mask = reinterpret_cast<unsigned long long*>(workspace);
  float* base = (float*)workspace + mask_floats;
  BwdWs w = bwd_ws(base, BN, 1, T, M);
  float* ht = base + w.floats;   // forward outputs of the mask recompute (unused)
  float* xt = ht + n * 64;
  float* vt = xt + n * 3;
  // the forward's LeakyReLU decisions, recomputed (the same kernel as the training forward)
  TconvArgs a{};
  a.BN = BN; a.T = T; a.M = M; a.Mfull = modes;
  a.h = h; a.x = x; a.v = v; a.lm = loc_mean; a.wp = tconv_blob; a.wx = tconvx_w;
  a.h_out = ht; a.x_out = xt; a.v_out = vt; a.frames = 0; a.mask_out = mask;
  if (int rc = launch_tconv(false, a, s)) return rc;
  const float *gx = g_x, *gv = g_v, *gh = g_h;
  if (!g_x) { hipMemsetAsync(w.gx[0], 0, n * 3 * sizeof(float), s); gx = w.gx[0]; }
  if (!g_v) { hipMemsetAsync(w.gv[0], 0, n * 3 * sizeof(float), s); gv = w.gv[0]; }
  if (!g_h) { hipMemsetAsync(w.gh[0], 0, n * 64 * sizeof(float), s); gh = w.gh[0]; }
  TconvRev tr;
  tr.BN = BN; tr.T = T; tr.M = M; tr.modes = modes; tr.frames = 0;
  tr.hs = h; tr.xs = x; tr.vs = v; tr.lm = loc_mean; tr.tw = tconv_w; tr.txw = tconvx_w; tr.mask = mask;
  tr.gh = gh; tr.gx = gx; tr.gv = gv;
  tr.g_hin = g_h_in; tr.g_xin = g_x_in; tr.g_vin = g_v_in; tr.g_tw = g_tconv_w; tr.g_txw = g_tconvx_w;
  return tconv_reverse(tr, w, s);
}

}  // extern "C"
