// nonode_bwd_common.h — shared by the training translation units (nonode_train.hip, included by
// nonode.hip, and nonode_node.hip): the backward weight-blob layout, true-scale SiLU helpers, the
// power-of-two column scaling of the fp16x3 gradient products, and the node-backward interface.
#pragma once
#include "nonode_common.h"

namespace {

// ---- backward weight blob (unscaled f32 fragments, forward and transposed) --------------------
enum : int {
  BOFF_WA = 0,          // edge W1 h_i columns                 (frag layout, KT=4)
  BOFF_WB = 4096,       // edge W1 h_j columns
  BOFF_W2 = 8192,       // edge W2
  BOFF_WC1 = 12288,     // coord W1
  BOFF_WV1 = 16384,     // node_v W1
  BOFF_WN1 = 20480,     // node W1 [64][128]                   (KT=8)
  BOFF_WN2 = 28672,     // node W2
  BOFF_W2T = 32768,     // W2^T
  BOFF_WC1T = 36864,    // Wc1^T
  BOFF_WV1T = 40960,    // WV1^T
  BOFF_WN2T = 45056,    // WN2^T
  BOFF_WN1TH = 49152,   // (WN1[:, 0:64])^T    (h columns)
  BOFF_WN1TM = 53248,   // (WN1[:, 64:128])^T  (message-sum columns)
  BOFF_WAT = 57344,     // W_A^T
  BOFF_WBT = 61440,     // W_B^T
  BOFF_FEAT = 65536,    // scalar-input columns [s, e...] as k-steps (as OFF_FEAT, unscaled)
  BOFF_VEC = 66048,     // vectors (vp order), BV_* below
};
enum : int { BV_B1 = 0, BV_B2, BV_BC1, BV_WC2, BV_BV1, BV_WV2, BV_BN1, BV_BN2, BV_WS, BV_COUNT };
constexpr int BOFF_SCAL = BOFF_VEC + BV_COUNT * 64;   // [0] coord b2, [1] node_v b2, [SC_*] option flags
// fp16 hi/lo fragments (pack_h16 layout, unscaled) of the 64x64 matrices: the edge backward's
// forward recompute (W2, Wc1), its transposed products (W2^T, Wc1^T) and its chunk tables
// P = W_A h + b1, Q = W_B h; the node backward's WV1, WN1 (h and message columns), their transposes
// and WN2^T (contiguous, in the order node_bwd_kernel stages them)
constexpr int BOFF_H16 = BOFF_SCAL + 64;
enum : int {
  BH_W2 = 0, BH_WC1, BH_W2T, BH_WC1T, BH_WA, BH_WB,
  BH_WV1, BH_WN1A, BH_WN1B, BH_WV1T, BH_WN2T, BH_WN1TH, BH_WN1TM, BH_WAT, BH_WBT, BH_COUNT
};
constexpr int BH_NODE0 = BH_WV1, BH_NODE_COUNT = BH_WN1TM + 1 - BH_WV1;   // node_bwd_kernel's seven
constexpr int BBLOB_FLOATS = BOFF_H16 + BH_COUNT * 4096;

// ---- true-scale SiLU and its derivative ---------------------------------------------------------
__device__ __forceinline__ float sigm(float z) { return __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(z * NEG_LOG2E)); }
__device__ __forceinline__ void silu_true(f4 (&a)[4]) {
#pragma unroll
  for (int mt = 0; mt < 4; ++mt)
#pragma unroll
    for (int q = 0; q < 4; ++q) a[mt][q] *= sigm(a[mt][q]);
}
// g *= silu'(z) = s (1 + z (1 - s))
__device__ __forceinline__ void mul_dsilu(f4 (&gz)[4], const f4 (&z)[4]) {
#pragma unroll
  for (int mt = 0; mt < 4; ++mt)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float s = sigm(z[mt][q]);
      gz[mt][q] *= s * fmaf(z[mt][q], 1.f - s, 1.f);
    }
}
__device__ __forceinline__ void zero4(f4 (&a)[4]) {
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) a[mt] = f4{0.f, 0.f, 0.f, 0.f};
}
// a = SiLU(z) keeping the sigmoid s for the reverse pass (one exp + one rcp per value, not two)
__device__ __forceinline__ void silu_keep(const f4 (&z)[4], f4 (&s)[4], f4 (&a)[4]) {
#pragma unroll
  for (int mt = 0; mt < 4; ++mt)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      s[mt][q] = sigm(z[mt][q]);
      a[mt][q] = z[mt][q] * s[mt][q];
    }
}
// a = SiLU(z) and d = SiLU'(z) = s (1 + z (1 - s)) (one exp + one rcp per value)
__device__ __forceinline__ void silu_dsilu(const f4 (&z)[4], f4 (&a)[4], f4 (&d)[4]) {
#pragma unroll
  for (int mt = 0; mt < 4; ++mt)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float s = sigm(z[mt][q]);
      a[mt][q] = z[mt][q] * s;
      d[mt][q] = s * fmaf(z[mt][q], 1.f - s, 1.f);
    }
}
// g *= silu'(z) from the kept sigmoid
__device__ __forceinline__ void mul_dsilu_s(f4 (&gz)[4], const f4 (&z)[4], const f4 (&s)[4]) {
#pragma unroll
  for (int mt = 0; mt < 4; ++mt)
#pragma unroll
    for (int q = 0; q < 4; ++q) gz[mt][q] *= s[mt][q] * fmaf(z[mt][q], 1.f - s[mt][q], 1.f);
}

// ---- fp16x3 products of the edge backward ----------------------------------------------------
// Activations are O(1) and take the forward's fp16x3 split (guarded by H16_LIMIT). Gradients have
// no fixed scale (they carry the loss normalisation, ~1e-7 here), so they are scaled by powers of
// two before the split: exact, and it keeps hi and lo out of the fp16 subnormal range.
// 2^(12 - e) for m = f 2^e (f in [0.5, 1)): m times it lies in [2^11, 2^12)
__device__ __forceinline__ float p2scale(float m) {
  int ex = __builtin_amdgcn_frexp_expf(m);
  ex = ex < -100 ? -100 : (ex > 100 ? 100 : ex);
  return __builtin_ldexpf(1.f, 12 - ex);
}
// max over the 4 lane groups (the 64 channels of column e)
__device__ __forceinline__ float col_max(float v) {
  const auto a = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = fmaxf(__uint_as_float(a[0]), __uint_as_float(a[1]));
  const auto b = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(b[0]), __uint_as_float(b[1]));
}
__device__ __forceinline__ float amax16(const f4 (&x)[4]) {
  float m[4];
#pragma unroll
  for (int mt = 0; mt < 4; ++mt)
    m[mt] = fmaxf(fmaxf(fabsf(x[mt][0]), fabsf(x[mt][1])), fmaxf(fabsf(x[mt][2]), fabsf(x[mt][3])));
  return fmaxf(fmaxf(m[0], m[1]), fmaxf(m[2], m[3]));
}
// max over the 16 lanes of a row (DPP: quad swaps, half-row and row mirrors; no LDS round trip)
template <int C>
__device__ __forceinline__ float dppf(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), C, 0xF, 0xF, false));
}
__device__ __forceinline__ float row_max16(float m) {
  m = fmaxf(m, dppf<0xB1>(m));    // quad_perm [1, 0, 3, 2]
  m = fmaxf(m, dppf<0x4E>(m));    // quad_perm [2, 3, 0, 1]
  m = fmaxf(m, dppf<0x141>(m));   // row_half_mirror
  return fmaxf(m, dppf<0x140>(m));  // row_mirror
}
// sum over the 16 lanes of a row (the same DPP steps: each adds a disjoint half, so every lane ends
// with the row's sum, in the same order on every lane)
__device__ __forceinline__ float row_sum16(float m) {
  m += dppf<0xB1>(m);
  m += dppf<0x4E>(m);
  m += dppf<0x141>(m);
  return m + dppf<0x140>(m);
}
// fp16x3 split of 4 values (as h16_split)
typedef _Float16 h4 __attribute__((ext_vector_type(4)));
typedef unsigned u2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void h4_split(f4 v, h4& hi, h4& lo) {
  hi = __builtin_convertvector(v, h4);
  const auto hw = __builtin_bit_cast(u2, hi);
  const f4 r = {resid_lo(hw[0], v[0]), resid_hi(hw[0], v[1]), resid_lo(hw[1], v[2]), resid_hi(hw[1], v[3])};
  lo = __builtin_convertvector(r, h4);
}
__device__ __forceinline__ float amax4(f4 v) {
  return fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fmaxf(fabsf(v[2]), fabsf(v[3])));
}
// fp16 images [32 rows][64 halves] read back transposed (ds_read_b64_tr_b16) as K = 32 MFMA operands:
// chunks of 8 halves XOR-swizzled per row (the edge backward's pair path and node_wgrad_kernel)
constexpr int IMG_HALVES = 32 * 64;   // one image (hi or lo): 32 rows x 64 halves
__device__ __forceinline__ int img_swz(int r) { return (((r >> 1) & 1) << 1) ^ ((r >> 2) & 1) ^ (((r >> 3) & 1) << 2); }
__device__ __forceinline__ int img_off(int r, int chunk) { return r * 64 + 8 * (chunk ^ img_swz(r)); }   // halves
typedef short s4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ h8 tr_read8(const _Float16* img, int t, int lane) {
  // lane 4q + p of group gq reads row 8 gq + q (+ 4), image columns 16 t + 4p .. + 3
  const int gq = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int c = 16 * t + 4 * p;                     // image column of the 4 halves
  const int r0 = 8 * gq + q, r1 = r0 + 4;
  const _Float16* a0 = img + img_off(r0, c >> 3) + (c & 7);
  const _Float16* a1 = img + img_off(r1, c >> 3) + (c & 7);
  const s4 v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s4*)(a0));
  const s4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s4*)(a1));
  typedef short s8 __attribute__((ext_vector_type(8)));
  const s8 v = {v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
  return __builtin_bit_cast(h8, v);
}
}  // namespace

namespace nonode_tu {
// ---- node backward (basic.py:174-185 reversed): nonode_node.hip --------------------------------
struct NodeBwdArgs {
  int n, N;
  const float* h; const float* v; const float* M; const float* F;   // layer inputs + saved sums
  const float* gxo; const float* gvo; const float* gho;              // grads of the layer outputs
  const float* bb;                                                   // backward blob
  float* gv; float* gF; float* gM; float* ghp;                       // outputs
  float* op_gt; float* op_z; float* op_gz;                           // GEMM operands (node_wgrad)
  float* p6;   // per-workgroup partials [blocks][65] of the node_v output row: sum gphi t | sum gphi
  float* GB; float* GX;                                              // zeroed for the edge backward
};
// launches node_bwd_kernel over ntile 16-node tiles on stream s (NONODE_OK or an error code); *nparts =
// the number of p6 partial rows it writes (at most NB_MAX_PARTS)
constexpr int NB_MAX_PARTS = 1024;
int launch_node_bwd(const NodeBwdArgs& a, int ntile, hipStream_t s, int* nparts);

// ---- gh = ghp + W_A^T GA + W_B^T GB, gx = gxo + GX after the edge backward (in node_wgrad_kernel) ----
struct NodePostArgs {
  int n;
  const float* ghp; const float* GA; const float* GB; const float* gxo; const float* GX;
  const float* bb;                 // backward blob (BH_WAT, BH_WBT fp16 fragments)
  float* gh; float* gx;
};

// ---- node-level weight gradients: nonode_node.hip ----------------------------------------------
// The layer's GEMMs over its n nodes, C_j = sum_k G_j[k] (x) A_j[k] (64x64, plus the bias column
// sum_k G_j[k]):
//   0 GA (x) h -> edge W1 h_i block (+ b1)    3 gz (x) h -> node W1 h block (+ b1)
//   1 GB (x) h -> edge W1 h_j block           4 gz (x) M -> node W1 message block
//   2 gt (x) h -> node_v W1 (+ b1)            5 gh (x) z -> node W2 (+ b2)
// (the node_v output row is node_bwd's, NodeBwdArgs::p6). Each workgroup writes one
// [NW_JOBS][64][65] partial; the caller adds them in block order (gemm_reduce_batch, deterministic).
// SEGNO (no node_v MLP) passes gt = null: job 2 is then zero.
constexpr int NW_JOBS = 6, NW_MAX_BLOCKS = 256, NW_PART = 64 * 65;
struct NodeWgradArgs {
  long long n, chunks_per_block;   // n nodes in 32-node chunks; block b takes chunks [b c, (b + 1) c)
  const float* h; const float* M; const float* z;                                      // A-side rows (n x 64)
  const float* GA; const float* GB; const float* gt; const float* gz; const float* gh;   // G-side rows
  float* partial;                                                                      // [blocks][NW_JOBS][NW_PART]
  NodePostArgs post;   // node_post fused (post.ghp non-null): gh = ghp + W_A^T GA + W_B^T GB from the staged GA / GB
};
// launches node_wgrad_kernel (returns the number of blocks, i.e. partials, in *nblk)
int launch_node_wgrad(const NodeWgradArgs& a, int* nblk, hipStream_t s);

constexpr int MMAX_T = 9;   // training path: every rfft bin of T <= 16 (as the forward, MMAX): tconv_bwd_kernel<1..9>

// ---- TimeConv reverse (layer_no.py:80-126; oracle/egno_grad.py spectral_bwd) -------------------
// Persistent: each 4-wave workgroup walks 16-column tiles (columns c = (b, n)). Per tile:
//   1. DFT of the input h (wave w: input channels 16w..16w+15) -> sX (the forward's layout);
//   2. (no forward recompute: the LeakyReLU decisions come from the forward, TrainState::mask);
//   3. gy[t] = gout[t] * leaky'(y[t]);  gYr_m = (c_m/T) sum_t cos gy,  gYi_m = -(c_m/T) sum_t sin gy
//      -> sG (zero for columns past BN);
//   4. backward mixing on MFMA: gXr = Wr gYr + Wi gYi, gXi = -Wi gYr + Wr gYi (wave w: input
//      channels 16w..) and gh[t] = gout[t] + sum_m (gXr_m cos - gXi_m sin)   (Xi = -sum_t h sin);
//   5. weight gradient: gWr_m += Xr (x) gYr + Xi (x) gYi,  gWi_m += -Xi (x) gYr + Xr (x) gYi over the
//      tile's columns (K = columns, read straight from sX / sG with channels along lane & 15),
//      wave w owning rows i = 16w..16w+15.
// One partial per workgroup [M][re|im][64][64]; tconv_wgrad_reduce adds them in a fixed order.
// A workgroup runs TB_NG(MM) such 4-wave groups on TB_NG tiles at once (own sX / sG, shared twiddles,
// the workgroup's barriers in lockstep): at C4 (640 tiles, 2 modes) every tile is in flight in one
// round instead of each CU walking 2-3 tiles one after another, a latency chain of load -> DFT ->
// barrier -> mixing -> store per tile. The groups' weight-gradient accumulators are added in group
// order before the one partial is written.

constexpr int TB_MAX_BLOCKS = 256;
// 4-wave tile groups per workgroup: two at <= 2 modes (three spill at the
// 170 registers of three waves per SIMD), else one
constexpr int tb_groups(int MM) { return MM <= 2 ? 2 : 1; }
struct TconvBwdArgs {
  int BN, T, M, ntiles;
  const float* h;      // TimeConv input [T][BN][64]
  const float* gout;   // gradient of its output
  const float* wb;     // backward fragments (tconv_pack_bwd_kernel layout)
  float* gh;           // gradient of the input
  float* wpart;        // [grid][M][2][64][64]
  const unsigned long long* mask;   // the forward's LeakyReLU decisions (TconvArgs::mask_out layout)
};

// launches tconv_bwd_kernel<M> (nonode_tconv.hip) on G workgroups
int launch_tconv_bwd(int M, TconvBwdArgs a, int G, hipStream_t s);
}  // namespace nonode_tu
