// EGNN_Layer with flat=True (EGNO main_simulation_simple_no.py --flat; basic.py:38-40: every BaseMLP
// 4x wide, 256 hidden channels, with Tanh): the forward (inference) on gfx950.
//
// Included at the end of nonode.hip (same translation unit: the ECL helpers, mfma_dense, the
// TimeConv and embedding launches). No BASELINE configuration uses flat=True, so this path is built
// for parity, not for speed: exact f32 MFMAs (v_mfma_f32_16x16x4_f32, mfma_dense) in three launches
// per layer, the 256-wide activations in registers in the ECL layout of 16 k-steps (lane (e, g) of
// column e holds channels 16 i + 4 g + q, i = 0..15, q = 0..3: the B operand of mfma_dense<16> and,
// block by block, the accumulators of four mfma_dense<KT> over 64-row slices).
//   flat_proj_kernel  P = W1[h_i] h + b1, Q = W1[h_j] h   (the edge MLP's first Linear, per node)
//   flat_edge_kernel  per receiver tile, all N-1 sender offsets: m = Tanh(W2 Tanh(P_i + Q_j +
//                     W1[s|e] [s, e]) + b2), c = wc2 . Tanh(Wc1 m + bc1) + bc2, f = r c; sums of m
//                     and f per receiver in registers (basic.py:167-173, aggregate basic.py:6-31)
//   flat_node_kernel  x += (wv2 . Tanh(Wv1 h + bv1) + bv2) v + clamp(mean f, +-100);
//                     h = Wn2 Tanh(Wn1 [h, sum m] + bn1) + bn2   (basic.py:174-185)

namespace {

// flat blob (floats): f32 MFMA A-operand fragments (pack_frag layout) and natural-order vectors
constexpr int FL_WA = 0;                  // W1[:, h_i columns]: 4 row blocks of 64 x (KT = 4)
constexpr int FL_WB = FL_WA + 4 * 4096;   // W1[:, h_j columns]
constexpr int FL_W2 = FL_WB + 4 * 4096;   // W2 [64][256]: KT = 16
constexpr int FL_WC1 = FL_W2 + 16384;     // Wc1 [256][64]: 4 row blocks, KT = 4
constexpr int FL_WV1 = FL_WC1 + 4 * 4096; // node_v W1 [256][64]
constexpr int FL_WN1 = FL_WV1 + 4 * 4096; // node W1 [256][128]: 4 row blocks, KT = 8
constexpr int FL_WN2 = FL_WN1 + 4 * 8192; // node W2 [64][256]: KT = 16
constexpr int FL_VEC = FL_WN2 + 16384;    // 256-wide vectors, FV_* below
enum : int { FV_B1 = 0, FV_WS, FV_WE0, FV_WE1, FV_WE2, FV_WE3, FV_BC1, FV_WC2, FV_BV1, FV_WV2, FV_BN1, FV_COUNT };
constexpr int FL_VEC64 = FL_VEC + FV_COUNT * 256;   // b2 [64], bn2 [64]
constexpr int FL_SCAL = FL_VEC64 + 128;             // [0] bc2, [1] bv2, [2] norm flag
constexpr int FL_FLOATS = FL_SCAL + 64;
constexpr int FL_EDGE_LDS = 2 * 16384;              // W2 and Wc1 fragments staged per workgroup

struct FlatPackArgs {
  const float *w1, *b1, *w2, *b2, *cw1, *cb1, *cw2, *cb2, *vw1, *vb1, *vw2, *vb2, *nw1, *nb1, *nw2, *nb2;
  int ld1, ne, norm;
  float* blob;
};
// one thread per blob float
__global__ void flat_pack_kernel(FlatPackArgs a) {
  const int d = blockIdx.x * blockDim.x + threadIdx.x;
  float* B = a.blob;
  if (d >= FL_FLOATS) return;
  if (d < FL_WB) {   // W1 h_i columns (EGNO order [s, h_i, h_j, e]: columns 1 .. 64)
    const int b = d >> 12;
    pack_frag(B + FL_WA + b * 4096, a.w1 + (size_t)64 * b * a.ld1, a.ld1, 1, 4, d & 4095, 1.f);
  } else if (d < FL_W2) {
    const int dd = d - FL_WB, b = dd >> 12;
    pack_frag(B + FL_WB + b * 4096, a.w1 + (size_t)64 * b * a.ld1, a.ld1, 1 + HID, 4, dd & 4095, 1.f);
  } else if (d < FL_WC1) {
    pack_frag(B + FL_W2, a.w2, 256, 0, 16, d - FL_W2, 1.f);
  } else if (d < FL_WV1) {
    const int dd = d - FL_WC1, b = dd >> 12;
    pack_frag(B + FL_WC1 + b * 4096, a.cw1 + 64 * 64 * b, 64, 0, 4, dd & 4095, 1.f);
  } else if (d < FL_WN1) {
    const int dd = d - FL_WV1, b = dd >> 12;
    pack_frag(B + FL_WV1 + b * 4096, a.vw1 + 64 * 64 * b, 64, 0, 4, dd & 4095, 1.f);
  } else if (d < FL_WN2) {
    const int dd = d - FL_WN1, b = dd >> 13;
    pack_frag(B + FL_WN1 + b * 8192, a.nw1 + 64 * 128 * b, 128, 0, 8, dd & 8191, 1.f);
  } else if (d < FL_VEC) {
    pack_frag(B + FL_WN2, a.nw2, 256, 0, 16, d - FL_WN2, 1.f);
  } else if (d < FL_VEC64) {
    const int v = (d - FL_VEC) >> 8, c = (d - FL_VEC) & 255;
    float val = 0.f;
    switch (v) {
      case FV_B1: val = a.b1[c]; break;
      case FV_WS: val = a.w1[(size_t)c * a.ld1]; break;   // the |r|^2 column
      case FV_WE0: case FV_WE1: case FV_WE2: case FV_WE3:
        val = (v - FV_WE0) < a.ne ? a.w1[(size_t)c * a.ld1 + 2 * HID + 1 + (v - FV_WE0)] : 0.f;
        break;
      case FV_BC1: val = a.cb1[c]; break;
      case FV_WC2: val = a.cw2[c]; break;
      case FV_BV1: val = a.vb1[c]; break;
      case FV_WV2: val = a.vw2[c]; break;
      case FV_BN1: val = a.nb1[c]; break;
    }
    B[d] = val;
  } else if (d < FL_SCAL) {
    const int c = d - FL_VEC64;
    B[d] = c < 64 ? a.b2[c] : a.nb2[c - 64];
  } else {
    const int i = d - FL_SCAL;
    B[d] = i == 0 ? a.cb2[0] : (i == 1 ? a.vb2[0] : (i == 2 ? (a.norm ? 1.f : 0.f) : 0.f));
  }
}

// lane's 64 values of a 256-wide natural-order vector / row, ECL-16 layout
__device__ __forceinline__ void load_ecl16(f4 (&d)[16], const float* row, int g) {
#pragma unroll
  for (int i = 0; i < 16; ++i) d[i] = *reinterpret_cast<const f4*>(row + 16 * i + 4 * g);
}
__device__ __forceinline__ void store_ecl16(float* row, const f4 (&s)[16], int g) {
#pragma unroll
  for (int i = 0; i < 16; ++i) *reinterpret_cast<f4*>(row + 16 * i + 4 * g) = s[i];
}
__device__ __forceinline__ void tanh16(f4 (&a)[16]) {
#pragma unroll
  for (int i = 0; i < 16; ++i)
#pragma unroll
    for (int q = 0; q < 4; ++q) a[i][q] = tanhf(a[i][q]);
}
// out (256 channels) += W x for a 256 x (16 KT) matrix stored as 4 row blocks of mfma_dense<KT> fragments
template <int KT>
__device__ __forceinline__ void mm256(f4 (&out)[16], const float* wf, const f4* in, int lane) {
#pragma unroll
  for (int b = 0; b < 4; ++b) {
    f4 acc[4] = {out[4 * b], out[4 * b + 1], out[4 * b + 2], out[4 * b + 3]};
    mfma_dense<KT>(acc, wf + b * 64 * 16 * KT, in, lane);
#pragma unroll
    for (int mo = 0; mo < 4; ++mo) out[4 * b + mo] = acc[mo];
  }
}
// sum over the 256 channels of w . a (w natural order): the lane's 64 products, then the 4 lane groups
__device__ __forceinline__ float dot256(const f4 (&a)[16], const float* w, int g) {
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const f4 wv = *reinterpret_cast<const f4*>(w + 16 * i + 4 * g);
#pragma unroll
    for (int q = 0; q < 4; ++q) s = fmaf(wv[q], a[i][q], s);
  }
  return group_sum(s);
}

struct FlatArgs {
  int n_total, n_graphs, N, ne, ef_mod;
  const float* h; const float* x; const float* v; const float* ef; const float* blob;
  float* P; float* Q; float* M; float* F;   // workspace [n][256], [n][256], [n][64], [n][4]
  float* h_out; float* x_out;
};

// P, Q rows of 16 nodes per wave
__global__ __launch_bounds__(256) void flat_proj_kernel(FlatArgs p) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, e = lane & 15, g = lane >> 4;
  const int r0 = (blockIdx.x * 4 + wave) * 16;
  if (r0 >= p.n_total) return;
  const int r = min(r0 + e, p.n_total - 1);
  f4 hin[4];
  load_ecl(hin, p.h + (size_t)r * HID, g);
  f4 acc[16];
  load_ecl16(acc, p.blob + FL_VEC + FV_B1 * 256, g);
  mm256<4>(acc, p.blob + FL_WA, hin, lane);
  if (r0 + e < p.n_total) store_ecl16(p.P + (size_t)r * 256, acc, g);
#pragma unroll
  for (int i = 0; i < 16; ++i) acc[i] = f4{0.f, 0.f, 0.f, 0.f};
  mm256<4>(acc, p.blob + FL_WB, hin, lane);
  if (r0 + e < p.n_total) store_ecl16(p.Q + (size_t)r * 256, acc, g);
}

// one wave per 16-receiver tile, every sender offset k = 1 .. N-1 in turn (receiver r meets sender
// (n + k) mod N of its graph); W2 / Wc1 fragments staged in LDS once per workgroup
__global__ __launch_bounds__(256) void flat_edge_kernel(FlatArgs p) {
  extern __shared__ __attribute__((aligned(16))) float fsm[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, e = lane & 15, g = lane >> 4;
  for (int i = tid; i < FL_EDGE_LDS / 4; i += 256)
    reinterpret_cast<f4*>(fsm)[i] = reinterpret_cast<const f4*>(p.blob + FL_W2)[i];   // W2 | Wc1 adjacent
  __syncthreads();
  const float* sW2 = fsm;
  const float* sWc1 = fsm + 16384;
  const float* vec = p.blob + FL_VEC;
  const float bc2 = p.blob[FL_SCAL + 0];
  const bool norm = p.blob[FL_SCAL + 2] != 0.f;
  const int N = p.N, Nm1 = N - 1;
  const int r0 = (blockIdx.x * 4 + wave) * 16;
  if (r0 >= p.n_total) return;
  const bool rvalid = r0 + e < p.n_total;
  const int r = rvalid ? r0 + e : p.n_total - 1;
  const int gr = r / N, n = r - gr * N;
  f4 Pr[16];
  load_ecl16(Pr, p.P + (size_t)r * 256, g);
  const float x0 = p.x[(size_t)r * 3 + 0], x1 = p.x[(size_t)r * 3 + 1], x2 = p.x[(size_t)r * 3 + 2];
  const float* efr = p.ef + ((size_t)(gr % p.ef_mod) * N + n) * Nm1 * p.ne;
  f4 Msum[4];
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) Msum[mt] = f4{0.f, 0.f, 0.f, 0.f};
  float F0 = 0.f, F1 = 0.f, F2 = 0.f;
#pragma unroll 1
  for (int k = 1; k < N; ++k) {
    int j = n + k;
    j = j >= N ? j - N : j;
    const int jj = j < n ? j : j - 1;
    const size_t s = (size_t)gr * N + j;
    const float q0 = x0 - p.x[s * 3 + 0], q1 = x1 - p.x[s * 3 + 1], q2 = x2 - p.x[s * 3 + 2];
    float sr = fmaf(q0, q0, fmaf(q1, q1, q2 * q2));
    if (norm) sr = radial_norm(sr);
    float fe[4] = {0.f, 0.f, 0.f, 0.f};
    for (int f = 0; f < p.ne; ++f) fe[f] = efr[(size_t)jj * p.ne + f];
    // a = Tanh(P_r + Q_s + W1[:, s] s + W1[:, e] e)
    f4 a[16];
    load_ecl16(a, p.Q + s * 256, g);
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int c = 16 * i + 4 * g;
      f4 t = Pr[i] + a[i] + *reinterpret_cast<const f4*>(vec + FV_WS * 256 + c) * sr;
#pragma unroll
      for (int f = 0; f < 4; ++f)
        if (f < p.ne) t += *reinterpret_cast<const f4*>(vec + (FV_WE0 + f) * 256 + c) * fe[f];
      a[i] = t;
    }
    tanh16(a);
    // m = Tanh(W2 a + b2)
    f4 m[4];
    load_ecl(m, p.blob + FL_VEC64, g);
    mfma_dense<16>(m, sW2, a, lane);
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int q = 0; q < 4; ++q) m[mt][q] = tanhf(m[mt][q]);
    // c = wc2 . Tanh(Wc1 m + bc1) + bc2
    f4 t[16];
    load_ecl16(t, vec + FV_BC1 * 256, g);
    mm256<4>(t, sWc1, m, lane);
    tanh16(t);
    const float c = dot256(t, vec + FV_WC2 * 256, g) + bc2;
    if (rvalid) {
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) Msum[mt] += m[mt];
      F0 = fmaf(q0, c, F0);
      F1 = fmaf(q1, c, F1);
      F2 = fmaf(q2, c, F2);
    }
  }
  if (rvalid) {
    store_ecl(p.M + (size_t)r * HID, Msum, g);
    if (g == 0) *reinterpret_cast<f4*>(p.F + (size_t)r * 4) = f4{F0, F1, F2, 0.f};
  }
}

// node update of 16 rows per wave
__global__ __launch_bounds__(256) void flat_node_kernel(FlatArgs p) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, e = lane & 15, g = lane >> 4;
  const int r0 = (blockIdx.x * 4 + wave) * 16;
  if (r0 >= p.n_total) return;
  const bool rvalid = r0 + e < p.n_total;
  const int r = rvalid ? r0 + e : p.n_total - 1;
  const float* vec = p.blob + FL_VEC;
  f4 in8[8];
  load_ecl(*reinterpret_cast<f4(*)[4]>(&in8[0]), p.h + (size_t)r * HID, g);
  load_ecl(*reinterpret_cast<f4(*)[4]>(&in8[4]), p.M + (size_t)r * HID, g);
  // phi = wv2 . Tanh(Wv1 h + bv1) + bv2 ;  x += phi v + clamp(mean f, +-100)
  f4 t[16];
  load_ecl16(t, vec + FV_BV1 * 256, g);
  mm256<4>(t, p.blob + FL_WV1, in8, lane);
  tanh16(t);
  const float phi = dot256(t, vec + FV_WV2 * 256, g) + p.blob[FL_SCAL + 1];
  // h = Wn2 Tanh(Wn1 [h, M] + bn1) + bn2
  load_ecl16(t, vec + FV_BN1 * 256, g);
  mm256<8>(t, p.blob + FL_WN1, in8, lane);
  tanh16(t);
  f4 hn[4];
  load_ecl(hn, p.blob + FL_VEC64 + 64, g);
  mfma_dense<16>(hn, p.blob + FL_WN2, t, lane);
  if (rvalid) {
    store_ecl(p.h_out + (size_t)r * HID, hn, g);
    if (g == 0) {
      const float inv = 1.f / (float)(p.N - 1);
      const f4 Fr = *reinterpret_cast<const f4*>(p.F + (size_t)r * 4);
#pragma unroll
      for (int d = 0; d < 3; ++d)
        p.x_out[(size_t)r * 3 + d] =
            p.x[(size_t)r * 3 + d] + phi * p.v[(size_t)r * 3 + d] + fminf(fmaxf(Fr[d] * inv, -100.f), 100.f);
    }
  }
}

// one flat EGNN layer: three launches (projections, edges, node update); ws = n x 580 floats
int launch_flat_layer(int n_graphs, int N, int ne, int ef_mod, const float* h, const float* x, const float* v,
                      const float* ef, const float* blob, float* h_out, float* x_out, float* ws, hipStream_t s) {
  static std::once_flag once;
  std::call_once(once, [] {
    hipFuncSetAttribute((const void*)flat_edge_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                        FL_EDGE_LDS * 4);
  });
  FlatArgs a;
  a.n_total = n_graphs * N; a.n_graphs = n_graphs; a.N = N; a.ne = ne; a.ef_mod = ef_mod;
  a.h = h; a.x = x; a.v = v; a.ef = ne ? ef : blob; a.blob = blob;
  const size_t n = (size_t)a.n_total;
  a.P = ws; a.Q = ws + n * 256; a.M = ws + n * 512; a.F = ws + n * 576;
  a.h_out = h_out; a.x_out = x_out;
  const int blocks = (int)((n + 63) / 64);
  hipLaunchKernelGGL(flat_proj_kernel, dim3(blocks), dim3(256), 0, s, a);
  if (int rc = check_launch("flat_proj_kernel")) return rc;
  hipLaunchKernelGGL(flat_edge_kernel, dim3(blocks), dim3(256), FL_EDGE_LDS * 4, s, a);
  if (int rc = check_launch("flat_edge_kernel")) return rc;
  hipLaunchKernelGGL(flat_node_kernel, dim3(blocks), dim3(256), 0, s, a);
  return check_launch("flat_node_kernel");
}

}  // namespace

extern "C" {

size_t nonode_flat_blob_floats(void) { return FL_FLOATS; }

int nonode_pack_layer_flat(const nonode_layer_weights* w, int variant, int hidden, int n_edge_feat, float* blob,
                           void* stream) {
  if (!w || !blob) return fail(NONODE_EINVAL, "pack_layer_flat: null pointer");
  const int flags = variant & ~0xff;
  if ((variant & 0xff) != NONODE_VARIANT_EGNO || (flags & ~NONODE_LAYER_NORM_RADIAL))
    return fail(NONODE_EINVAL, "pack_layer_flat: EGNO layers only (option bits 0x%x)", flags);
  if (hidden != HID || n_edge_feat < 0 || n_edge_feat > 4)
    return fail(NONODE_EUNSUPPORTED, "pack_layer_flat: hidden=%d n_edge_feat=%d", hidden, n_edge_feat);
  if (!w->edge_w1 || !w->edge_b1 || !w->edge_w2 || !w->edge_b2 || !w->coord_w1 || !w->coord_b1 || !w->coord_w2 ||
      !w->coord_b2 || !w->vel_w1 || !w->vel_b1 || !w->vel_w2 || !w->vel_b2 || !w->node_w1 || !w->node_b1 ||
      !w->node_w2 || !w->node_b2)
    return fail(NONODE_EINVAL, "pack_layer_flat: missing weight pointer");
  FlatPackArgs a{w->edge_w1, w->edge_b1, w->edge_w2, w->edge_b2, w->coord_w1, w->coord_b1, w->coord_w2, w->coord_b2,
                 w->vel_w1, w->vel_b1, w->vel_w2, w->vel_b2, w->node_w1, w->node_b1, w->node_w2, w->node_b2,
                 2 * HID + 1 + n_edge_feat, n_edge_feat, (flags & NONODE_LAYER_NORM_RADIAL) ? 1 : 0, blob};
  hipLaunchKernelGGL(flat_pack_kernel, dim3((FL_FLOATS + 255) / 256), dim3(256), 0, (hipStream_t)stream, a);
  return check_launch("flat_pack_kernel");
}

}  // extern "C"
