// nonode_node.hip — the node side of the EGNO backward (basic.py:174-185 reversed), its own
// translation unit: built with the default machine scheduler, because the iterative-ILP scheduler
// that nonode.hip is built with leaves invalid live intervals in this kernel's fp16x3 form (machine
// verifier: "No live segment at use"; LLVM's greedy register allocator then crashes).
#include "nonode_bwd_common.h"

namespace {

using nonode_tu::NodeBwdArgs;

// column-scaled fp16x3 split of a 16-column operand (as mm64_cs); returns the inverse scale
__device__ __forceinline__ float cs_split(const f4 (&x)[4], h8 (&xh)[2], h8 (&xl)[2]) {
  const float sc = p2scale(col_max(amax16(x)));
  f4 xs[4];
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) xs[mt] = x[mt] * sc;
  h16_split(xs, xh, xl);
  return 1.f / sc;   // exact (power of two)
}
// out (+)= inv * W x (W: one staged fragment set)
template <bool ADD>
__device__ __forceinline__ void mm_node(f4 (&out)[4], const h8* wh, const h8 (&xh)[2], const h8 (&xl)[2],
                                        float inv, int lane, unsigned us) {
  f4 acc[4];
  zero4(acc);
  mfma_h16(acc, wh, xh, xl, lane, us);
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) out[mt] = ADD ? out[mt] + acc[mt] * inv : acc[mt] * inv;
}
// ---- node_bwd_kernel (NodeBwdArgs) ---------------------------------------------------------------
// Persistent: one workgroup (8 waves, two per SIMD) per CU stages the node-side matrices in LDS once
// (112 KB) and its waves walk 16-node tiles. (One tile per wave with the fragments read from L2 moved
// ~128 KB of fragments per 16 nodes: 92 us per C4 layer, L2-bound.) Also zeroes the edge backward's
// GB / GX rows.
constexpr int NB_WAVES = 8;
// The seven products (WV1 h, WN1 [h, M], WV1^T gt, WN2^T gho, WN1^T gz) run fp16x3 on
// v_mfma_f32_16x16x32_f16 (24 MFMAs each, against 64 or 128 f32 16x16x4 MFMAs of 4x the cycles):
// every operand column is scaled by a power of two to [2^11, 2^12) before the split and the product
// scaled back (cs_split, exact), so activations and gradients of any magnitude take the same path.
constexpr int NB_LDS_FLOATS = BH_NODE_COUNT * 4096;   // 28672: the seven fp16 hi/lo fragment sets
__global__ __launch_bounds__(NB_WAVES * 64) void node_bwd_kernel(NodeBwdArgs p) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, e = lane & 15, g = lane >> 4;
  {
    const f4* src = reinterpret_cast<const f4*>(p.bb + BOFF_H16 + BH_NODE0 * 4096);
    for (int i = threadIdx.x; i < NB_LDS_FLOATS / 4; i += NB_WAVES * 64) reinterpret_cast<f4*>(smem)[i] = src[i];
  }
  __syncthreads();
  const h8* sH_ = reinterpret_cast<const h8*>(smem);
  const int ntile = (p.n + 15) >> 4;
  // the node_v output row's gradient sum_n gphi_n t_n (and sum_n gphi_n), per lane: column e's terms
  // for channels 16 mt + 4 g + q; the wave's 16 columns are added at the end (no t / gphi to HBM)
  f4 s6[4];
  zero4(s6);
  float b6 = 0.f;
#pragma unroll 1
  for (int tile = blockIdx.x * NB_WAVES + wave; tile < ntile; tile += gridDim.x * NB_WAVES) {
  // loop-invariant reads stay in the loop (hoisted, the 7 x 64 fragment registers per lane would
  // not fit): opaque zero offset
  int off = 0;
  asm volatile("" : "+v"(off));
  const float* bb = p.bb + off;
  const h8* sH = sH_ + off;
  const auto W = [&](int k) { return sH + (k - BH_NODE0) * 1024; };
  const auto us = [&](int k) { return h16_us(bb + BOFF_SCAL, k); };
  const int r0 = tile * 16;
  const int r = min(r0 + e, p.n - 1);
  const bool valid = r0 + e < p.n;
  f4 hr[4], Mr[4];
  load_ecl(hr, p.h + (size_t)r * HID, g);
  load_ecl(Mr, p.M + (size_t)r * HID, g);
  h8 xh[2], xl[2];
  float inv = cs_split(hr, xh, xl);
  // phi_v(h) = wv2 . SiLU(WV1 h + bv1) + bv2;  node MLP pre-activation zp = WN1 [h, M] + bn1
  f4 tp[4], zp[4];
  load_vp(tp, bb + BOFF_VEC + BV_BV1 * 64, g);
  mm_node<true>(tp, W(BH_WV1), xh, xl, inv, lane, us(BH_WV1));
  load_vp(zp, bb + BOFF_VEC + BV_BN1 * 64, g);
  mm_node<true>(zp, W(BH_WN1A), xh, xl, inv, lane, us(BH_WN1A));
  inv = cs_split(Mr, xh, xl);
  mm_node<true>(zp, W(BH_WN1B), xh, xl, inv, lane, us(BH_WN1B));
  f4 t[4];
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) t[mt] = tp[mt];
  silu_true(t);
  const float phi = dot_vp(t, bb + BOFF_VEC + BV_WV2 * 64, g) + bb[BOFF_SCAL + 1];
  const float gx0 = p.gxo[(size_t)r * 3 + 0], gx1 = p.gxo[(size_t)r * 3 + 1], gx2 = p.gxo[(size_t)r * 3 + 2];
  const float v0 = p.v[(size_t)r * 3 + 0], v1 = p.v[(size_t)r * 3 + 1], v2 = p.v[(size_t)r * 3 + 2];
  const float gphi = gx0 * v0 + gx1 * v1 + gx2 * v2;
  // clamp(F / (N-1), +-100) passes the gradient inside [-100, 100]
  const float finv = 1.f / (float)(p.N - 1);
  const float F0 = p.F[(size_t)r * 4 + 0] * finv, F1 = p.F[(size_t)r * 4 + 1] * finv, F2 = p.F[(size_t)r * 4 + 2] * finv;
  const float gF0 = (F0 >= -100.f && F0 <= 100.f) ? gx0 * finv : 0.f;
  const float gF1 = (F1 >= -100.f && F1 <= 100.f) ? gx1 * finv : 0.f;
  const float gF2 = (F2 >= -100.f && F2 <= 100.f) ? gx2 * finv : 0.f;
  // gt_pre = gphi * wv2 (.) silu'(tp);  gh = WV1^T gt_pre
  f4 gt[4];
  load_vp(gt, bb + BOFF_VEC + BV_WV2 * 64, g);
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) gt[mt] *= gphi;
  mul_dsilu(gt, tp);
  f4 gh[4];
  inv = cs_split(gt, xh, xl);
  mm_node<false>(gh, W(BH_WV1T), xh, xl, inv, lane, us(BH_WV1T));
  // node MLP reverse: gz = WN2^T gho (.) silu'(zp), gh += WN1h^T gz, gM = WN1m^T gz
  f4 z[4];
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) z[mt] = zp[mt];
  silu_true(z);
  f4 gho[4], gz[4];
  load_ecl(gho, p.gho + (size_t)r * HID, g);
  inv = cs_split(gho, xh, xl);
  mm_node<false>(gz, W(BH_WN2T), xh, xl, inv, lane, us(BH_WN2T));
  mul_dsilu(gz, zp);
  inv = cs_split(gz, xh, xl);
  mm_node<true>(gh, W(BH_WN1TH), xh, xl, inv, lane, us(BH_WN1TH));
  f4 gM[4];
  mm_node<false>(gM, W(BH_WN1TM), xh, xl, inv, lane, us(BH_WN1TM));
  if (valid) {
    const size_t o = (size_t)r * HID;
    store_ecl(p.ghp + o, gh, g);
    store_ecl(p.gM + o, gM, g);
    store_ecl(p.op_gt + o, gt, g);
    store_ecl(p.op_z + o, z, g);
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) s6[mt] += t[mt] * gphi;
    b6 += gphi;
    store_ecl(p.op_gz + o, gz, g);
    const f4 z4[4] = {};
    store_ecl(p.GB + o, z4, g);                          // the edge backward's sender sums start at 0
    if (g == 0) {
      p.gv[(size_t)r * 3 + 0] = p.gvo[(size_t)r * 3 + 0] + phi * gx0;
      p.gv[(size_t)r * 3 + 1] = p.gvo[(size_t)r * 3 + 1] + phi * gx1;
      p.gv[(size_t)r * 3 + 2] = p.gvo[(size_t)r * 3 + 2] + phi * gx2;
      *reinterpret_cast<f4*>(p.gF + (size_t)r * 4) = f4{gF0, gF1, gF2, 0.f};
      *reinterpret_cast<f4*>(p.GX + (size_t)r * 4) = f4{0.f, 0.f, 0.f, 0.f};
    }
  }
  }
  // the wave's 16 columns added (DPP row sums: lanes 16 g + e, e = 0..15), then the block's 8 waves in
  // wave order through LDS (the fragments' space): one partial row per workgroup
  __syncthreads();
  float* srow = smem + wave * 68;
#pragma unroll
  for (int mt = 0; mt < 4; ++mt)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float v = row_sum16(s6[mt][q]);
      if (e == 0) srow[16 * mt + 4 * g + q] = v;
    }
  const float bt = row_sum16(b6);
  if (lane == 0) srow[64] = bt;
  __syncthreads();
  if (threadIdx.x < 65) {
    float v = 0.f;
#pragma unroll
    for (int w = 0; w < NB_WAVES; ++w) v += smem[w * 68 + threadIdx.x];
    p.p6[(size_t)blockIdx.x * 65 + threadIdx.x] = v;
  }
}


// ---- node-level weight gradients (NodeWgradArgs) ------------------------------------------------
// One 12-wave workgroup per CU walks its range of 32-node chunks. Each chunk's nine operand slabs
// (32 x 64 floats each) are staged in LDS once (row stride 80 floats: the 64 lanes of an MFMA operand
// read hit 64 distinct banks), so HBM sees every operand row once (the unfused form read h four times
// and gz twice). Wave w accumulates rows [32 (w & 1), +32) of GEMM w >> 1 with exact f32 MFMAs
// (v_mfma_f32_16x16x4_f32: the products of the reference's fp32 autograd GEMMs, summed in a fixed
// order), three waves per SIMD; the next chunk's rows are loaded into registers while the current one
// is multiplied. node_post runs here too (NodeWgradArgs::post, waves 0..3), on the staged GA / GB: the
// separate kernel read GA, GB again (26 us per C4 layer).
constexpr int NW_WAVES = 12, NW_CH = 32, NW_ROW = 80, NW_SLABS = 9;
constexpr int NW_SLAB = NW_CH * NW_ROW;                                   // floats per staged slab
constexpr int NW_LDS_FLOATS = NW_SLABS * NW_SLAB;
constexpr int NW_LDS_POST = 2 * 4096;                                    // W_A^T | W_B^T fp16 hi/lo (fused node_post)
// output rows [32 hf, +32) of W x (one fragment set), hf = 0 / 1: 12 of mfma_h16's 24 MFMAs, same chains
__device__ __forceinline__ void mfma_h16_half(f4 (&acc)[2], const h8* wf, const h8 (&xh)[2], const h8 (&xl)[2],
                                              int lane, unsigned us, int hf) {
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    h8 ah[2], al[2];
#pragma unroll
    for (int m = 0; m < 2; ++m) {
      ah[m] = wf[((s * 4 + 2 * hf + m) * 2 + 0) * 64 + lane];
      al[m] = wf[((s * 4 + 2 * hf + m) * 2 + 1) * 64 + lane];
    }
    const h8 xs = h8_scale(xh[s], us);
#pragma unroll
    for (int m = 0; m < 2; ++m) acc[m] = mfma16(ah[m], xh[s], acc[m]);
#pragma unroll
    for (int m = 0; m < 2; ++m) acc[m] = mfma16(al[m], xs, acc[m]);
#pragma unroll
    for (int m = 0; m < 2; ++m) acc[m] = mfma16(ah[m], xl[s], acc[m]);
  }
}
constexpr int NW_SLAB_F4 = NW_CH * 16;                                   // f4 loads per slab (512)
__global__ __launch_bounds__(NW_WAVES * 64) void node_wgrad_kernel(nonode_tu::NodeWgradArgs p) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, il = lane & 15, kg = lane >> 4;
  // slab order: h, M, z (A side), ghp (node_post's addend), GA, GB, gt, gz, gh (G side)
  const float* const src[NW_SLABS] = {p.h, p.M, p.z, p.post.ghp, p.GA, p.GB, p.gt, p.gz, p.gh};
  float* sG = smem;                                 // [slab][node][NW_ROW]
  const h8* sWp = reinterpret_cast<const h8*>(smem + NW_LDS_FLOATS);   // fused node_post fragments
  const bool post = p.post.ghp != nullptr;
  if (post) {
    const f4* wsrc = reinterpret_cast<const f4*>(p.post.bb + BOFF_H16 + BH_WAT * 4096);   // W_A^T | W_B^T
    for (int i = tid; i < NW_LDS_POST / 4; i += NW_WAVES * 64) reinterpret_cast<f4*>(smem + NW_LDS_FLOATS)[i] = wsrc[i];
  }
  const int job = wave >> 1, a0 = 2 * (wave & 1);
  constexpr int GS[6] = {4, 5, 6, 7, 7, 8}, AS[6] = {0, 0, 0, 0, 1, 2};
  const int gslab = GS[job], aslab = AS[job];
  const bool active = job != 2 || p.gt != nullptr;   // wave-uniform (SEGNO: no node_v MLP, job 2 idle)
  const long long c0 = (long long)blockIdx.x * p.chunks_per_block;
  long long c1 = c0 + p.chunks_per_block;
  const long long nch = (p.n + NW_CH - 1) / NW_CH;
  c1 = c1 < nch ? c1 : nch;
  f4 acc[2][4];
  float bsum[2] = {0.f, 0.f};
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = f4{0.f, 0.f, 0.f, 0.f};
  // register prefetch of one chunk: threads tid < 512 load f4 (node tid >> 4, channels 4 (tid & 15) ..)
  // of every slab (the slab loop is unrolled, so each source pointer is a kernel argument)
  f4 pre[NW_SLABS];
  const int pnode = (tid >> 4) & 31, pc4 = tid & 15;
  auto fetch = [&](long long c) {
    const long long row = c * NW_CH + pnode;
    const bool ok = tid < NW_SLAB_F4 && row < p.n;
    long long off = row * 64 + 4 * pc4;
    asm volatile("" : "+v"(off));   // (one offset, not nine hoisted per-thread source pointers)
#pragma unroll
    for (int sl = 0; sl < NW_SLABS; ++sl)   // (a null source: SEGNO has no gt, zeros)
      pre[sl] = (ok && src[sl]) ? *reinterpret_cast<const f4*>(src[sl] + off) : f4{0.f, 0.f, 0.f, 0.f};
  };
  if (c0 < c1) fetch(c0);
#pragma unroll 1
  for (long long c = c0; c < c1; ++c) {
    __syncthreads();   // every wave is done with the previous chunk
    if (tid < NW_SLAB_F4) {
#pragma unroll
      for (int sl = 0; sl < NW_SLABS; ++sl)
        *reinterpret_cast<f4*>(sG + sl * NW_SLAB + pnode * NW_ROW + 4 * pc4) = pre[sl];
    }
    __syncthreads();
    // node_post (before the next chunk's prefetch, whose registers it reuses): waves 0..3 (one per
    // SIMD) take tile wave >> 1 of the chunk, output rows [32 (wave & 1), +32); gh = (ghp + A) + B
    if (post && wave < 4) {
      const int tl = wave >> 1, hf = wave & 1;
      int off = 0;   // (keeps the loop-invariant fragment reads in the loop, see node_bwd_kernel)
      asm volatile("" : "+v"(off));
      const long long row = c * NW_CH + 16 * tl + il;
      const bool ok = row < p.n;
      f4 o[2];
#pragma unroll
      for (int m = 0; m < 2; ++m)
        o[m] = *reinterpret_cast<const f4*>(sG + 3 * NW_SLAB + (16 * tl + il) * NW_ROW + 16 * (2 * hf + m) + 4 * kg);
#pragma unroll
      for (int pr = 0; pr < 2; ++pr) {   // GA (slab 4) through W_A^T, GB (slab 5) through W_B^T
        const float* xr = sG + (4 + pr) * NW_SLAB + (16 * tl + il) * NW_ROW;
        f4 x[4];
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) x[mt] = *reinterpret_cast<const f4*>(xr + 16 * mt + 4 * kg);
        h8 xh[2], xl[2];
        const float inv = cs_split(x, xh, xl);
        f4 a[2] = {f4{0.f, 0.f, 0.f, 0.f}, f4{0.f, 0.f, 0.f, 0.f}};
        mfma_h16_half(a, sWp + off + pr * 1024, xh, xl, lane, h16_us(p.post.bb + BOFF_SCAL, pr ? BH_WBT : BH_WAT), hf);
#pragma unroll
        for (int m = 0; m < 2; ++m) o[m] = o[m] + a[m] * inv;
      }
      if (ok) {
#pragma unroll
        for (int m = 0; m < 2; ++m) *reinterpret_cast<f4*>(p.post.gh + row * 64 + 16 * (2 * hf + m) + 4 * kg) = o[m];
        if (hf == 0 && kg < 3) p.post.gx[row * 3 + kg] = p.post.gxo[row * 3 + kg] + p.post.GX[row * 4 + kg];
      }
    }
    if (c + 1 < c1) fetch(c + 1);
    const float* g = sG + gslab * NW_SLAB;
    const float* av = sG + aslab * NW_SLAB;
#pragma unroll
    for (int kk = 0; kk < (active ? NW_CH / 4 : 0); ++kk) {
      const int node = 4 * kk + kg;
      float gv[2], xv[4];
#pragma unroll
      for (int a = 0; a < 2; ++a) gv[a] = g[node * NW_ROW + 16 * (a0 + a) + il];
#pragma unroll
      for (int b = 0; b < 4; ++b) xv[b] = av[node * NW_ROW + 16 * b + il];
#pragma unroll
      for (int a = 0; a < 2; ++a) {
        bsum[a] += gv[a];
#pragma unroll
        for (int b = 0; b < 4; ++b) acc[a][b] = mfma(gv[a], xv[b], acc[a][b]);
      }
    }
  }
  // partials: this block's [job][64][65]
  float* out = p.partial + (size_t)blockIdx.x * nonode_tu::NW_JOBS * nonode_tu::NW_PART;
  float* oj = out + (size_t)job * nonode_tu::NW_PART;
#pragma unroll
  for (int a = 0; a < 2; ++a) {
#pragma unroll
    for (int b = 0; b < 4; ++b)
#pragma unroll
      for (int q = 0; q < 4; ++q) oj[(16 * (a0 + a) + 4 * kg + q) * 65 + 16 * b + il] = acc[a][b][q];
    const float bs = group_sum(bsum[a]);
    if (kg == 0) oj[(16 * (a0 + a) + il) * 65 + 64] = bs;
  }
}
}  // namespace

namespace nonode_tu {
int launch_node_bwd(const NodeBwdArgs& a, int ntile, hipStream_t s, int* nparts) {
  static std::once_flag once;
  std::call_once(once, [] {
    hipFuncSetAttribute((const void*)node_bwd_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, NB_LDS_FLOATS * 4);
  });
  const int want = (ntile + NB_WAVES - 1) / NB_WAVES;
  int G = want < num_cus() ? want : num_cus();
  G = G < NB_MAX_PARTS ? G : NB_MAX_PARTS;
  if (G < 1) G = 1;
  *nparts = G;
  hipLaunchKernelGGL(node_bwd_kernel, dim3(G), dim3(NB_WAVES * 64), NB_LDS_FLOATS * 4, s, a);
  return check_launch("node_bwd_kernel");
}

int launch_node_wgrad(const NodeWgradArgs& a_in, int* nblk, hipStream_t s) {
  static std::once_flag once;
  std::call_once(once, [] {
    hipFuncSetAttribute((const void*)node_wgrad_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                        (NW_LDS_FLOATS + NW_LDS_POST) * 4);
  });
  NodeWgradArgs a = a_in;
  const long long nch = (a.n + NW_CH - 1) / NW_CH;
  long long G = num_cus();
  G = G < NW_MAX_BLOCKS ? G : NW_MAX_BLOCKS;
  G = nch < G ? nch : G;
  if (G < 1) G = 1;
  a.chunks_per_block = (nch + G - 1) / G;
  G = (nch + a.chunks_per_block - 1) / a.chunks_per_block;
  if (G < 1) G = 1;
  *nblk = (int)G;
  const int lds = (NW_LDS_FLOATS + (a.post.ghp ? NW_LDS_POST : 0)) * 4;
  hipLaunchKernelGGL(node_wgrad_kernel, dim3((unsigned)G), dim3(NW_WAVES * 64), lds, s, a);
  return check_launch("node_wgrad_kernel");
}

}  // namespace nonode_tu
