// vn_policy.hip — goal-conditioned CNN policy (BigGoalHouseModel trunk + heads) forward
// and backward in fp32 on MFMA, gfx950.
//
// Reference topology (models/goal.py:36-59, 77-92):
//   shared_base: Conv(3->32, k7 s4) ReLU, Conv(32->32, k4 s2) ReLU   — image and goal, shared weights
//   concat(image, goal) on channels                                   — goal.py:88
//   conv_base:  Conv(64->64, k4 s2) ReLU, Conv(64->32, k1) ReLU
//   conv_merge: Flatten, Linear(32*h3*w3 -> 512), ReLU                — in_features derived from the frame
//   heads:      policy_logits Linear(512->A), critic Linear(512->1)   — fused into one [A+1 x 512] head
// Layout: activations NHWC fp32, samples contiguous, frame f = 2*sample + {0: image, 1: goal};
// weights [Cout][ky][kx][Cin] (K padded to a multiple of 4) + bias. conv_merge runs as a
// 3x3 "conv" over the 3x3x32 map (its torch weight [512][c*9+y*3+x] is permuted on load).
// Inputs: uint8 HWC frames gathered straight from the scene cache by row index (the
// env never has to materialise the batch), converted x = u8/255 as ScaledFloatFrame does.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <mutex>
#include <new>
#include <map>
#include <tuple>
#include <unordered_map>

#include "vn_common.h"
#include "vn_gemm.h"
#include "vn_lstm.h"
#include "vn_aux.h"
#include "vn_unreal.h"
#include "vn_skinny.h"

#include "vn_frames.h"
#include "vn_conv1.h"
namespace vn {

// ---- operand loaders ---------------------------------------------------------
// conv1 im2col over 3-channel frames; k = (ky*7 + kx)*3 + c, K = 147 (padded 148).
template <int H, int W, int OH, int OW>
struct FramesIm2col {
  FrameSrc src;
  int M;  // 2 * samples * OH * OW
  __device__ __forceinline__ f4 load4(int m, int k, int kend) const {
    f4 v = f4zero();
    if (m >= M) return v;
    const int f = m / (OH * OW);
    const int r = m - f * (OH * OW);
    const int oy = r / OW, ox = r - (r / OW) * OW;
    const int smp = f >> 1, h = f & 1;
    const int lim = min(kend, 147);
    if (src.f32[h]) {
      const float* fr = src.f32[h] + (int64_t)smp * 3 * H * W;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int kk = k + j;
        if (kk < lim) {
          const int ky = kk / 21, kx = (kk / 3) % 7, c = kk % 3;
          v[j] = fr[((int64_t)c * H + oy * 4 + ky) * W + ox * 4 + kx];
        }
      }
    } else {
      const int64_t row = src.rows[h] ? (int64_t)src.rows[h][smp] : (int64_t)smp;
      const uint8_t* fr = src.base[h] + row * src.stride;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int kk = k + j;
        if (kk < lim) {
          const int ky = kk / 21, kx = (kk / 3) % 7, c = kk % 3;
          v[j] = (float)fr[((oy * 4 + ky) * W + ox * 4 + kx) * 3 + c] / 255.0f;
        }
      }
    }
    return v;
  }
  VN_ROWS_LOADER
};

// im2col over NHWC fp32 with G channel-concatenated input groups (C % 4 == 0).
template <int C, int KH, int KW, int S, int H, int W, int OH, int OW, int G>
struct NhwcIm2col {
  const float* X;
  int M;  // samples * OH * OW
  __device__ __forceinline__ f4 load4(int m, int k, int kend) const {
    if (m >= M || k >= kend) return f4zero();
    const int n = m / (OH * OW);
    const int r = m - n * (OH * OW);
    const int oy = r / OW, ox = r - (r / OW) * OW;
    const int c = k % C;
    int t = k / C;
    const int g = t % G;
    t /= G;
    const int ky = t / KW, kx = t % KW;
    return *reinterpret_cast<const f4*>(X + ((((int64_t)n * G + g) * H + oy * S + ky) * W + ox * S + kx) * C + c);
  }
  VN_ROWS_LOADER
};

// conv3's im2col over concat(image, goal) X2 with goal-frame deduplication: group 1 (the goal
// map) of sample n is read from sample n + gd[n] (the start of its goal run, vn_goal_runs).
//
// As the A operand (conv3's forward) a thread's fetch slots keep their rows across the K loop,
// so the redirected sample of each slot is loaded once, at the first fetch, and kept in
// registers (a per-element gd load put a dependent load in front of every K tile's gather:
// +23 % per 174x174 call); as a transposed wgrad operand (rows = pixels, changing every K tile)
// load4 looks gd up per element.
template <int C, int KH, int KW, int S, int H, int W, int OH, int OW>
struct NhwcIm2colGoal {
  static constexpr int kMaxSlots = 8;
  const float* X;
  int M;  // samples * OH * OW
  const int32_t* gd;
  mutable int gsm[kMaxSlots];  // slot j's goal sample (first fetch)
  mutable bool ready;
  __device__ __forceinline__ f4 load_at(int m, int k, int kend, int64_t ngoal) const {
    if (m >= M || k >= kend) return f4zero();
    const int n = m / (OH * OW);
    const int r = m - n * (OH * OW);
    const int oy = r / OW, ox = r - (r / OW) * OW;
    const int c = k % C;
    int t = k / C;
    const int g = t & 1;
    t >>= 1;
    const int ky = t / KW, kx = t % KW;
    const int64_t ns = g ? ngoal : (int64_t)n;
    return *reinterpret_cast<const f4*>(X + (((ns * 2 + g) * H + oy * S + ky) * W + ox * S + kx) * C + c);
  }
  __device__ __forceinline__ f4 load4(int m, int k, int kend) const {
    const int n = m < M ? m / (OH * OW) : 0;
    return load_at(m, k, kend, (int64_t)n + gd[n]);
  }
  static constexpr bool kTrans = false;
  template <int ROWS, int BK>
  static constexpr int slots() { return ROWS * (BK / 4); }
  template <int ROWS, int BK>
  __device__ __forceinline__ void fetch(f4* r, int row0, int k0, int kend, int tid) const {
    constexpr int Q = BK / 4, T = ROWS * Q, NS = (T + 255) / 256;
    static_assert(NS <= kMaxSlots, "fetch slots");
    if (!ready) {
#pragma unroll
      for (int j = 0; j < NS; ++j) {
        int rr, q;
        rows_slot<ROWS, Q>(tid + j * 256, rr, q);
        const int m = row0 + rr;
        const int n = m < M ? m / (OH * OW) : 0;
        gsm[j] = n + gd[n];
      }
      ready = true;
    }
#pragma unroll
    for (int j = 0; j < NS; ++j) {
      const int i = tid + j * 256;
      if (T % 256 == 0 || i < T) {
        int rr, q;
        rows_slot<ROWS, Q>(i, rr, q);
        r[j] = load_at(row0 + rr, k0 + 4 * q, kend, gsm[j]);
      }
    }
  }
  template <int ROWS, int BK, int LD>
  __device__ __forceinline__ static void commit(const f4* r, float* s, int tid) {
    commit_rows<ROWS, BK, LD>(r, s, tid);
  }
};

// conv3's forward A operand (NhwcIm2colGoal's rows and values) with the gather's addressing
// taken out of the K loop: with BK == C a K tile is one (g, ky, kx) — uniform — so each fetch
// slot keeps the offsets of its image and goal patches (computed at the first fetch, in 16-B
// units from X: a goal run's start can lie gigabytes back in an earlier call's samples) and a
// K tile adds one uniform offset. Rows past M read row 0's patch: the epilogue stores no row
// past M, so they need no zeros. The per-slot row decomposition, bounds tests and address math
// of the generic gather (~16 vector instructions per slot and K tile) become a select and a
// 64-bit add. gd == nullptr: each sample's own goal half (NhwcIm2col<..., G = 2>'s rows).
// Requires BK == C and K % BK == 0 (conv3: K = 1024).
template <int C, int KH, int KW, int S, int H, int W, int OH, int OW>
struct NhwcIm2colGoalF {
  static constexpr int kMaxSlots = 8;
  const float* X;
  int M;  // samples * OH * OW
  const int32_t* gd;
  mutable int oimg[kMaxSlots], ogoal[kMaxSlots];
  mutable bool ready;
  static constexpr bool kTrans = false;
  template <int ROWS, int BK>
  static constexpr int slots() { return ROWS * (BK / 4); }
  template <int ROWS, int BK>
  __device__ __forceinline__ void fetch(f4* r, int row0, int k0, int kend, int tid) const {
    static_assert(BK == C && C % 4 == 0, "one (g, ky, kx) per K tile");
    constexpr int Q = BK / 4, T = ROWS * Q, NS = (T + 255) / 256;
    static_assert(NS <= kMaxSlots, "fetch slots");
    (void)kend;
    if (!ready) {
#pragma unroll
      for (int j = 0; j < NS; ++j) {
        int rr, q;
        rows_slot<ROWS, Q>(tid + j * 256, rr, q);
        const int m = row0 + rr < M ? row0 + rr : 0;
        const int n = m / (OH * OW);
        const int rm = m - n * (OH * OW);
        const int oy = rm / OW, ox = rm - (rm / OW) * OW;
        const int base = (((oy * S) * W + ox * S) * C + 4 * q) / 4;
        oimg[j] = (2 * n) * (H * W * C / 4) + base;
        ogoal[j] = (2 * (n + (gd ? gd[n] : 0)) + 1) * (H * W * C / 4) + base;
      }
      ready = true;
    }
    int t = k0 / C;
    const bool g = t & 1;
    t >>= 1;
    const int ky = t / KW, kx = t - (t / KW) * KW;
    const f4* xb = reinterpret_cast<const f4*>(X) + (ky * W + kx) * (C / 4);
#pragma unroll
    for (int j = 0; j < NS; ++j)
      if (T % 256 == 0 || tid + j * 256 < T) r[j] = xb[g ? ogoal[j] : oimg[j]];
  }
};

// conv2's im2col (one 32-channel input, k4 s2) over the frames of a FrameList (goal-frame
// deduplication on maps without a persistent conv2 kernel, 300x400): row m = (list item
// m / (OH*OW), output pixel); rows end at the list's device-side count (row_limit).
template <int H, int W, int OH, int OW>
struct FrameListIm2col {
  const float* X;
  int M;  // host upper bound: 2 * samples * OH * OW
  FrameList fl;
  __device__ __forceinline__ int row_limit() const { return fl_count(fl, 0) * (OH * OW); }
  __device__ __forceinline__ f4 load4(int m, int k, int kend) const {
    if (m >= M || k >= kend) return f4zero();
    const int i = m / (OH * OW);
    const int r = m - i * (OH * OW);
    const int oy = r / OW, ox = r - (r / OW) * OW;
    const int c = k & 31, t = k >> 5, ky = t >> 2, kx = t & 3;
    const int64_t f = fl_frame_v(fl, i);
    return *reinterpret_cast<const f4*>(X + ((f * H + oy * 2 + ky) * W + ox * 2 + kx) * 32 + c);
  }
  VN_ROWS_LOADER
};

// Bias + ReLU into the listed frames' maps (row m of FrameListIm2col -> its frame's pixel).
template <int OH, int OW>
struct EpiBiasActFrames {
  float* Y;
  const float* bias;
  FrameList fl;
  __device__ __forceinline__ float pre_col(int col) const { return bias[col]; }
  __device__ __forceinline__ void post(int row, int col, float v, float b, int) const {
    const int i = row / (OH * OW), r = row - i * (OH * OW);
    Y[((int64_t)fl_frame_v(fl, i) * (OH * OW) + r) * 32 + col] = fmaxf(v + b, 0.0f);
  }
};

// BigHouseModel conv1 (Conv2d(3, 32, k8, s4), bignet.py:29) im2col over the image frame
// only: row m = (sample, oy, ox), k = (ky*8 + kx)*3 + c, K = 192; u8 frames as x/255
// (ScaledFloatFrame) or dense float NCHW frames.
template <int H, int W, int OH, int OW>
struct FramesIm2colK8 {
  FrameSrc src;
  int M;  // samples * OH * OW
  __device__ __forceinline__ f4 load4(int m, int k, int kend) const {
    f4 v = f4zero();
    if (m >= M) return v;
    const int smp = m / (OH * OW);
    const int r = m - smp * (OH * OW);
    const int oy = r / OW, ox = r - (r / OW) * OW;
    const int lim = min(kend, 192);
    if (src.f32[0]) {
      const float* fr = src.f32[0] + (int64_t)smp * 3 * H * W;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int kk = k + j;
        if (kk < lim) {
          const int ky = kk / 24, kx = (kk / 3) % 8, c = kk % 3;
          v[j] = fr[((int64_t)c * H + oy * 4 + ky) * W + ox * 4 + kx];
        }
      }
    } else {
      const int64_t row = src.rows[0] ? (int64_t)src.rows[0][smp] : (int64_t)smp;
      const uint8_t* fr = src.base[0] + row * src.stride;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int kk = k + j;
        if (kk < lim) {
          const int ky = kk / 24, kx = (kk / 3) % 8, c = kk % 3;
          v[j] = (float)fr[((oy * 4 + ky) * W + ox * 4 + kx) * 3 + c] / 255.0f;
        }
      }
    }
    return v;
  }
  VN_ROWS_LOADER
};

// Dense row-major matrix [rows][ld] (ld % 4 == 0, 16-B aligned).
struct DenseRows {
  const float* A;
  int64_t ld;
  int M;
  __device__ __forceinline__ f4 load4_fast(int m, int k) const {
    return *reinterpret_cast<const f4*>(A + (int64_t)m * ld + k);
  }
  __device__ __forceinline__ f4 load4(int m, int k, int kend) const {
    if (m >= M || k >= kend) return f4zero();
    const float* p = A + (int64_t)m * ld + k;
    if (k + 3 < kend) return *reinterpret_cast<const f4*>(p);
    f4 v = f4zero();
    for (int j = 0; j < 4 && k + j < kend; ++j) v[j] = p[j];
    return v;
  }
  VN_ROWS_LOADER
};

// Row-major rows [0, M) of A plus a ones row at m == M (k < kend): the transposed input
// of a row-fill wgrad, whose ones row gives the bias gradient column.
struct RowsOnes {
  const float* A;
  int64_t ld;
  int M;
  __device__ __forceinline__ f4 load4_fast(int m, int k) const {
    return *reinterpret_cast<const f4*>(A + (int64_t)m * ld + k);
  }
  __device__ __forceinline__ f4 load4(int m, int k, int kend) const {
    if (m > M || k >= kend) return f4zero();
    f4 v = f4zero();
    if (m == M) {
      for (int j = 0; j < 4 && k + j < kend; ++j) v[j] = 1.0f;
      return v;
    }
    const float* p = A + (int64_t)m * ld + k;
    if (k + 3 < kend) return *reinterpret_cast<const f4*>(p);
    for (int j = 0; j < 4 && k + j < kend; ++j) v[j] = p[j];
    return v;
  }
  VN_ROWS_LOADER
};

// wgrad A operand: dZ [P][ld] read as rows r..r+3 (output channels) at pixel p.
struct DenseT {
  const float* A;
  int64_t ld;
  int ncols;
  __device__ __forceinline__ f4 load4t(int p, int r) const {
    const float* q = A + (int64_t)p * ld + r;
    if (r + 3 < ncols) return *reinterpret_cast<const f4*>(q);
    f4 v = f4zero();
    for (int j = 0; j < 4 && r + j < ncols; ++j) v[j] = q[j];
    return v;
  }
  VN_TRANS_LOADER
};

// wgrad B operand over dense rows read transposed: X [P][ld] as rows r..r+3 (columns of X) at
// pixel p, plus a ones row at r == ncols (that column of the product is the bias gradient).
struct DenseTOnes {
  const float* A;
  int64_t ld;
  int ncols;
  __device__ __forceinline__ f4 load4t(int p, int r) const {
    const float* q = A + (int64_t)p * ld + r;
    if (r + 3 < ncols) return *reinterpret_cast<const f4*>(q);
    f4 v = f4zero();
    for (int j = 0; j < 4; ++j) v[j] = r + j < ncols ? q[j] : (r + j == ncols ? 1.0f : 0.0f);
    return v;
  }
  VN_TRANS_LOADER
};

// wgrad B operand: an im2col loader read transposed, plus a ones column at k == KP
// (that column of the product is the bias gradient).
template <class L>
struct Im2colT {
  L l;
  int KP;
  __device__ __forceinline__ f4 load4t(int p, int r) const {
    f4 v = l.load4(p, r, KP);
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (r + j == KP) v[j] = 1.0f;
    return v;
  }
  VN_TRANS_LOADER
};

// dgrad of a strided conv, one (group g, parity py, px) class per launch: rows are the
// input pixels y = yy*S + py, x = xx*S + px; k = (tky, tkx, co) over the KH/S x KW/S taps
// that reach them (ky = py + tky*S, oy = yy - tky).
template <int COUT, int KW, int S, int OH, int OW, int HYC, int WXC>
struct DgradA {
  const float* dZ;
  int M;
  __device__ __forceinline__ f4 load4(int m, int k, int kend) const {
    if (m >= M || k >= kend) return f4zero();
    constexpr int per = HYC * WXC;
    const int n = m / per;
    const int r = m - n * per;
    const int yy = r / WXC, xx = r - (r / WXC) * WXC;
    const int co = k % COUT;
    const int t = k / COUT;
    const int tky = t / (KW / S), tkx = t % (KW / S);
    const int oy = yy - tky, ox = xx - tkx;
    if (oy < 0 || oy >= OH || ox < 0 || ox >= OW) return f4zero();
    return *reinterpret_cast<const f4*>(dZ + (((int64_t)n * OH + oy) * OW + ox) * COUT + co);
  }
  VN_ROWS_LOADER
};

template <int COUT, int KW, int S, int CINF>
struct DgradB {
  const float* WT;  // [KH*KW*CINF][COUT]
  int cin, g_off, py, px;
  __device__ __forceinline__ f4 load4(int j, int k, int kend) const {
    if (j >= cin || k >= kend) return f4zero();
    const int co = k % COUT;
    const int t = k / COUT;
    const int ky = py + (t / (KW / S)) * S, kx = px + (t % (KW / S)) * S;
    return *reinterpret_cast<const f4*>(WT + ((int64_t)(ky * KW + kx) * CINF + g_off + j) * COUT + co);
  }
  VN_ROWS_LOADER
};

// ---- epilogues ----------------------------------------------------------------
struct EpiBiasAct {
  float* Y;
  int64_t ld;
  const float* bias;
  int relu;
  __device__ __forceinline__ float pre_col(int col) const { return bias[col]; }
  __device__ __forceinline__ void post(int row, int col, float v, float b, int) const {
    v += b;
    Y[(int64_t)row * ld + col] = relu ? fmaxf(v, 0.0f) : v;
  }
};

// dX masked by the ReLU that produced X (X = relu(z) -> dz = dX * [X > 0]); may alias X.
struct EpiMask {
  float* out;
  const float* X;
  int64_t ld;
  __device__ __forceinline__ float pre(int row, int col) const { return X[(int64_t)row * ld + col]; }
  __device__ __forceinline__ void post(int row, int col, float v, float x, int) const {
    out[(int64_t)row * ld + col] = x > 0.0f ? v : 0.0f;
  }
};

template <int H, int W, int S, int PY, int PX, int HYC, int WXC>
struct EpiMaskParity {
  float* out;
  const float* X;
  int g, G, cin;
  __device__ __forceinline__ int64_t index(int row, int col) const {
    constexpr int per = HYC * WXC;
    const int n = row / per;
    const int r = row - n * per;
    const int y = (r / WXC) * S + PY, x = (r % WXC) * S + PX;
    return ((((int64_t)n * G + g) * H + y) * W + x) * cin + col;
  }
  __device__ __forceinline__ float pre(int row, int col) const { return X[index(row, col)]; }
  __device__ __forceinline__ void post(int row, int col, float v, float x, int) const {
    out[index(row, col)] = x > 0.0f ? v : 0.0f;
  }
};

// EpiMaskParity over all G channel groups at once: column c of the product is channel
// c % CIN of group c / CIN (input layout [n][G][H][W][CIN]).
template <int H, int W, int S, int PY, int PX, int HYC, int WXC, int CIN>
struct EpiMaskParityG {
  float* out;
  const float* X;
  int G;
  int mask_goal = 1;  // 0: group 1 unmasked (goal runs: masked at the run start by goal_dz2_reduce_kernel)
  __device__ __forceinline__ int64_t index(int row, int col) const {
    constexpr int per = HYC * WXC;
    const int n = row / per;
    const int r = row - n * per;
    const int y = (r / WXC) * S + PY, x = (r % WXC) * S + PX;
    return ((((int64_t)n * G + col / CIN) * H + y) * W + x) * CIN + col % CIN;
  }
  __device__ __forceinline__ float pre(int row, int col) const { return X[index(row, col)]; }
  __device__ __forceinline__ void post(int row, int col, float v, float x, int) const {
    out[index(row, col)] = (x > 0.0f || (!mask_goal && col >= CIN)) ? v : 0.0f;
  }
};

struct EpiSlab {
  float* slab;
  int M, N;
  __device__ __forceinline__ void operator()(int row, int col, float v, int z) const {
    slab[((int64_t)z * M + row) * N + col] = v;
  }
};

// A one-slab wgrad's epilogue: dW [M][KP] and the bias column into db (and db2), as
// wgrad_reduce_kernel writes them (its sum 0 + v, kept: -0 stores as +0), without the slab
// round trip and the reduce launch (a few-row backward ran eight of them, 7 us each).
struct EpiWgrad {
  float* dW;
  float* db;
  float* db2;
  int KP;
  __device__ __forceinline__ void operator()(int row, int col, float v, int) const {
    const float s = 0.0f + v;
    if (col < KP) {
      dW[(int64_t)row * KP + col] = s;
    } else {
      db[row] = s;
      if (db2) db2[row] = s;
    }
  }
};

// Split-K slab [splits][M][N] -> dW [M][KP] and, when N == KP + 1, the bias column db [M]
// (also into db2 when given: the LSTM's b_ih and b_hh share one gradient).
__global__ void wgrad_reduce_kernel(const float* __restrict__ slab, int splits, int M, int N, int KP, float* dW,
                                    float* db, float* db2) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= M * N) return;
  const int row = idx / N, col = idx - (idx / N) * N;
  float s = 0.0f;
  for (int z = 0; z < splits; ++z) s += slab[((int64_t)z * M + row) * N + col];
  if (col < KP)
    dW[(int64_t)row * KP + col] = s;
  else {
    db[row] = s;
    if (db2) db2[row] = s;
  }
}

// The same sum with G lanes per output (few outputs, many slabs: the one-thread form above ran
// 100-230 dependent loads per thread on 10-40 workgroups, 30-60 us): lane j of output idx sums
// slabs z = j (mod G) in order, then a fixed xor tree over the G lanes. Deterministic.
template <int G>
__global__ __launch_bounds__(256) void wgrad_reduce_g_kernel(const float* __restrict__ slab, int splits, int M, int N,
                                                             int KP, float* dW, float* db, float* db2) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t MN = (int64_t)M * N;
  const int64_t idx = t / G;
  const int j = (int)(t - idx * G);
  float s = 0.0f;
  if (idx < MN)
    for (int z = j; z < splits; z += G) s += slab[(int64_t)z * MN + idx];
#pragma unroll
  for (int o = G / 2; o > 0; o >>= 1) s += __shfl_xor(s, o);
  if (j != 0 || idx >= MN) return;
  const int row = (int)(idx / N), col = (int)(idx - (int64_t)row * N);
  if (col < KP)
    dW[(int64_t)row * KP + col] = s;
  else {
    db[row] = s;
    if (db2) db2[row] = s;
  }
}

// Launch the reduce of `splits` slabs of M x N partials: one thread per output while that
// fills the chip, else G lanes per output (about 8 slabs per lane).
inline void launch_wgrad_reduce(const float* slab, int splits, int M, int N, int KP, float* dW, float* db, float* db2,
                                hipStream_t st) {
  const int64_t MN = (int64_t)M * N;
  int G = 1;
  if (MN < 65536)
    while (G < 64 && G * 8 < splits) G *= 2;
  const unsigned blocks = (unsigned)((MN * G + 255) / 256);
  switch (G) {
    case 1: hipLaunchKernelGGL(wgrad_reduce_kernel, dim3(blocks), dim3(256), 0, st, slab, splits, M, N, KP, dW, db, db2); break;
    case 2: hipLaunchKernelGGL(wgrad_reduce_g_kernel<2>, dim3(blocks), dim3(256), 0, st, slab, splits, M, N, KP, dW, db, db2); break;
    case 4: hipLaunchKernelGGL(wgrad_reduce_g_kernel<4>, dim3(blocks), dim3(256), 0, st, slab, splits, M, N, KP, dW, db, db2); break;
    case 8: hipLaunchKernelGGL(wgrad_reduce_g_kernel<8>, dim3(blocks), dim3(256), 0, st, slab, splits, M, N, KP, dW, db, db2); break;
    case 16: hipLaunchKernelGGL(wgrad_reduce_g_kernel<16>, dim3(blocks), dim3(256), 0, st, slab, splits, M, N, KP, dW, db, db2); break;
    case 32: hipLaunchKernelGGL(wgrad_reduce_g_kernel<32>, dim3(blocks), dim3(256), 0, st, slab, splits, M, N, KP, dW, db, db2); break;
    default: hipLaunchKernelGGL(wgrad_reduce_g_kernel<64>, dim3(blocks), dim3(256), 0, st, slab, splits, M, N, KP, dW, db, db2); break;
  }
}

__global__ void transpose_kernel(const float* __restrict__ W, int rows, int cols, float* __restrict__ WT) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= rows * cols) return;
  const int r = idx / cols, c = idx - (idx / cols) * cols;
  WT[(int64_t)c * rows + r] = W[idx];
}

// Up to kTSet weight transposes WT[c][r] = W[r][c] in one launch, 64 x 64 tiles through LDS
// (reads and writes row-contiguous): workgroup b finds its matrix by a scan of the tile-range
// starts. A backward transposes its weights once (5 matrices of the trunk, 2 of the LSTM
// core); one launch each cost a dependent dispatch apiece on the few-env path, and the former
// element-wise map wrote one 4-byte value per 64-byte line (12 us per set at 4 envs).
constexpr int kTSet = 6;
struct TransposeSet {
  const float* W[kTSet];
  float* WT[kTSet];
  int rows[kTSet], cols[kTSet];
  int tstart[kTSet + 1];  // tile-range starts
  int n = 0;
  void add(const float* w, int r, int c, float* wt) {
    if ((int64_t)r * c == 0) return;
    if (n == 0) tstart[0] = 0;
    W[n] = w;
    WT[n] = wt;
    rows[n] = r;
    cols[n] = c;
    tstart[n + 1] = tstart[n] + ((r + 63) / 64) * ((c + 63) / 64);
    ++n;
  }
};

__global__ __launch_bounds__(256) void transpose_set_kernel(TransposeSet s) {
  __shared__ float t[64][65];
  const int b = blockIdx.x;
  int i = 0;
  while (i + 1 < s.n && b >= s.tstart[i + 1]) ++i;
  const int rows = s.rows[i], cols = s.cols[i], tc = (cols + 63) / 64, l = b - s.tstart[i];
  const int r0 = (l / tc) * 64, c0 = (l - (l / tc) * tc) * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const float* src = s.W[i];
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int r = r0 + ty + 4 * k, c = c0 + tx;
    if (r < rows && c < cols) t[ty + 4 * k][tx] = src[(int64_t)r * cols + c];
  }
  __syncthreads();
  float* dst = s.WT[i];
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int c = c0 + ty + 4 * k, r = r0 + tx;
    if (r < rows && c < cols) dst[(int64_t)c * rows + r] = t[tx][ty + 4 * k];
  }
}

inline void launch_transpose_set(const TransposeSet& s, hipStream_t st) {
  if (s.n == 0) return;
  hipLaunchKernelGGL(transpose_set_kernel, dim3((unsigned)s.tstart[s.n]), dim3(256), 0, st, s);
}

// dst[c][r] = src[r][c] for a rows x cols block (row strides lds / ldd), 64 x 64 tiles
// through LDS: both the reads and the writes are row-contiguous.
__global__ __launch_bounds__(256) void tile_transpose_kernel(const float* __restrict__ src, int rows, int cols,
                                                             int64_t lds, float* __restrict__ dst, int64_t ldd) {
  __shared__ float t[64][65];
  const int r0 = blockIdx.y * 64, c0 = blockIdx.x * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int r = r0 + ty + 4 * i, c = c0 + tx;
    if (r < rows && c < cols) t[ty + 4 * i][tx] = src[(int64_t)r * lds + c];
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int c = c0 + ty + 4 * i, r = r0 + tx;
    if (r < rows && c < cols) dst[(int64_t)c * ldd + r] = t[tx][ty + 4 * i];
  }
}

inline void tile_transpose(const float* src, int rows, int cols, int64_t lds, float* dst, int64_t ldd,
                           hipStream_t st) {
  hipLaunchKernelGGL(tile_transpose_kernel, dim3((cols + 63) / 64, (rows + 63) / 64), dim3(256), 0, st, src, rows, cols,
                     lds, dst, ldd);
}

// ---- geometry & layout ------------------------------------------------------------
struct LayerOff {
  int64_t w, b;
  int cout, kp;
};

struct PolicyLayout {
  int arch;  // 0: BigGoalHouseModel (goal.py), 1: BigHouseModel (bignet.py: image only, Nature-CNN trunk)
  int H, W, A, OH1, OW1, OH2, OW2, OH3, OW3, FCIN;
  LayerOff l[6];  // conv1, conv2, conv3, conv4, fc, head
  int64_t n_params;
  int64_t sz[5];  // per-sample floats of X1..X5
  int64_t msz;    // per-sample words of the conv1 ReLU bitmask (one uint32 of channel bits per pixel)
  int64_t wt_off[6], wt_total;
  // recurrent core (BigGoalHouseModel, models/goal.py:61-67): W_cat [2048][xcat] = [W_ih | 0 | W_hh]
  int lstm, lin, xoff, xcat;
  int64_t lw, lbih, lbhh;
  // aux deconv heads (AuxiliaryBigGoalHouseModel, goal.py:144-189): W1 [32][4][4][48], b1 [48],
  // W2 [48][4][4][8] (block diagonal), b2 [8]; maps X4 [h3][w3] -> A1 [AH][AW] -> P [PH][PW]
  int aux, AH, AW, PH, PW;
  int64_t aw1, ab1, aw2, ab2;
  // UNREAL heads (goal.py:94-133, vn_unreal.h): pc_base W [2592][512] (rows (y, x, c)), b [2592];
  // pc W1 [32][4][4][64], b1 [64]; pc W2 [64][4][4][8] (block diagonal), b2 [8]; rp W [3][3 FCIN], b [4]
  int unreal;
  int64_t upw, upb, uw1, ub1, uw2, ub2, urw, urb;
  // split-K scratch on the policy's device (vn_policy_create_ex): slabs of the products whose
  // tiles alone cannot fill the chip (small batches), see launch_gemm_x6_sk
  float* sk;
  int64_t sk_cap;  // floats
  int sk_dev;
};

inline PolicyLayout make_layout(int H, int W, int A, int lstm = 0, int aux = 0, int arch = 0, int unreal = 0) {
  PolicyLayout L{};
  L.arch = arch;
  L.H = H;
  L.W = W;
  L.A = A;
  if (arch == 1) {  // bignet.py:28-41: Conv(3,32,k8,s4), Conv(32,64,k4,s2), Conv(64,32,k3), Linear(32*7*7)
    L.OH1 = (H - 8) / 4 + 1;
    L.OW1 = (W - 8) / 4 + 1;
    L.OH2 = (L.OH1 - 4) / 2 + 1;
    L.OW2 = (L.OW1 - 4) / 2 + 1;
    L.OH3 = L.OH2 - 2;
    L.OW3 = L.OW2 - 2;
  } else {
    L.OH1 = (H - 7) / 4 + 1;
    L.OW1 = (W - 7) / 4 + 1;
    L.OH2 = (L.OH1 - 4) / 2 + 1;
    L.OW2 = (L.OW1 - 4) / 2 + 1;
    L.OH3 = (L.OH2 - 4) / 2 + 1;
    L.OW3 = (L.OW2 - 4) / 2 + 1;
  }
  L.FCIN = 32 * L.OH3 * L.OW3;
  const int couts_g[6] = {32, 32, 64, 32, 512, A + 1};
  const int ks_g[6] = {148, 16 * 32, 16 * 64, 64, L.FCIN, 512};
  const int couts_b[6] = {32, 64, 32, 0, 512, A + 1};  // layer 3 (conv4) absent
  const int ks_b[6] = {192, 16 * 32, 9 * 64, 0, L.FCIN, 512};
  const int* couts = arch == 1 ? couts_b : couts_g;
  const int* ks = arch == 1 ? ks_b : ks_g;
  int64_t off = 0, wt = 0;
  for (int i = 0; i < 6; ++i) {
    L.l[i].cout = couts[i];
    L.l[i].kp = ks[i];
    L.l[i].w = off;
    off += (int64_t)couts[i] * ks[i];
    L.l[i].b = off;
    off += couts[i];
    L.wt_off[i] = wt;
    if (i > 0) wt += (int64_t)couts[i] * ks[i];
  }
  L.lstm = lstm;
  L.lin = 512 + A + 1;
  L.xoff = (L.lin + 3) / 4 * 4;
  L.xcat = L.xoff + 512;
  if (lstm) {
    L.lw = off;
    off += 2048ll * L.xcat;
    L.lbih = off;
    off += 2048;
    L.lbhh = off;
    off += 2048;
  }
  L.aux = aux;
  L.AH = 2 * L.OH3 + 2;
  L.AW = 2 * L.OW3 + 2;
  L.PH = 2 * L.AH + 2;
  L.PW = 2 * L.AW + 2;
  if (aux) {
    L.aw1 = off;
    off += 32ll * 16 * kAuxC1;
    L.ab1 = off;
    off += kAuxC1;
    L.aw2 = off;
    off += (int64_t)kAuxC1 * 16 * kAuxC2;
    L.ab2 = off;
    off += kAuxC2;
  }
  L.unreal = unreal;
  if (unreal) {
    off = (off + 3) / 4 * 4;  // float4 rows for the products
    L.upw = off;
    off += (int64_t)kPcBase * 512;
    L.upb = off;
    off += kPcBase;
    // BigHouseModel (bignet.py:77-91): one transposed conv per branch, 32 -> 8 (value 0..A-1,
    // action A, padding) in W1 / b1; no second layer (W2, b2 empty)
    const int c1 = arch == 1 ? kPcC2 : kPcC1;
    L.uw1 = off;
    off += 32ll * 16 * c1;
    L.ub1 = off;
    off += c1;
    L.uw2 = off;
    if (arch != 1) off += (int64_t)kPcC1 * 16 * kPcC2;
    L.ub2 = off;
    if (arch != 1) off += kPcC2;
    L.urw = off;
    off += 3ll * 3 * L.FCIN;
    L.urb = off;
    off += 4;
  }
  L.n_params = off;
  L.wt_total = wt;
  if (arch == 1) {  // X1 (one frame per sample), X2, X3, no X4, X5; no ReLU bitmask
    L.sz[0] = (int64_t)L.OH1 * L.OW1 * 32;
    L.sz[1] = (int64_t)L.OH2 * L.OW2 * 64;
    L.sz[2] = (int64_t)L.OH3 * L.OW3 * 32;
    L.sz[3] = 0;
    L.sz[4] = 512;
    L.msz = 0;
    return L;
  }
  L.sz[0] = 2ll * L.OH1 * L.OW1 * 32;
  L.sz[1] = 2ll * L.OH2 * L.OW2 * 32;
  L.sz[2] = (int64_t)L.OH3 * L.OW3 * 64;
  L.sz[3] = (int64_t)L.OH3 * L.OW3 * 32;
  L.sz[4] = 512;
  L.msz = 2ll * L.OH1 * L.OW1;
  return L;
}

constexpr int OUT_LD = 8;  // [n][8]: logits 0..A-1, value at A
constexpr int kConv1WgradBlocks = 512;  // x 4 wave slabs x 32 x 160 floats (fits the slab)
constexpr int kConv2WgradBlocks = 512;  // x (32 x 512 + 32) floats (fits the slab)

// Resident workgroups of a persistent kernel on the current device, cached per (device,
// kernel, threads, LDS bytes): a process may drive policies on several devices.
inline int resident_blocks(const void* kernel, int threads, size_t lds) {
  static std::mutex mu;
  static std::map<std::tuple<int, const void*, int, size_t>, int> cache;
  int dev = 0, cus = 0, per = 0;
  (void)hipGetDevice(&dev);
  std::lock_guard<std::mutex> lock(mu);
  const auto key = std::make_tuple(dev, kernel, threads, lds);
  auto it = cache.find(key);
  if (it != cache.end()) return it->second;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kernel, threads, lds) != hipSuccess || per < 1) per = 1;
  if (getenv("VN_DEBUG_OCC")) {
    hipFuncAttributes fa{};
    (void)hipFuncGetAttributes(&fa, kernel);
    fprintf(stderr, "[vn occ] kernel %p threads %d lds %zu: %d blocks/CU (numRegs %d, static lds %zu)\n", kernel,
            threads, lds, per, fa.numRegs, (size_t)fa.sharedSizeBytes);
  }
  const int blocks = std::max(1, per * std::max(cus, 1));
  cache[key] = blocks;
  return blocks;
}

// Opt-in to `lds` bytes of dynamic LDS for `kernel` on the current device, once per (device,
// kernel) and again only if a larger size is asked for (the attribute is per device).
inline hipError_t ensure_dyn_lds(const void* kernel, size_t lds) {
  static std::mutex mu;
  static std::map<std::pair<int, const void*>, size_t> done;
  int dev = 0;
  (void)hipGetDevice(&dev);
  std::lock_guard<std::mutex> lock(mu);
  size_t& have = done[std::make_pair(dev, kernel)];
  if (have >= lds) return hipSuccess;
  const hipError_t e = hipFuncSetAttribute(kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e == hipSuccess) have = lds;
  return e;
}

inline dim3 grid_for(int M, int N, int BM, int BN, int splits = 1) {
  return dim3((M + BM - 1) / BM, (N + BN - 1) / BN, splits);
}

template <int BM, int BN, int BK, int WM, int WN, class FA, class FB, class EP>
inline void launch_gemm(FA fa, FB fb, EP ep, int M, int N, int K, hipStream_t st, int splits = 1, int kchunk = 0) {
  if (M <= 0 || N <= 0) return;
  if (kchunk <= 0) kchunk = K;
  hipLaunchKernelGGL((gemm_kernel<BM, BN, BK, WM, WN, FA, FB, EP>), grid_for(M, N, BM, BN, splits), dim3(256), 0,
                     st, fa, fb, ep, M, N, K, kchunk);
}

template <int BM, int BN, int BK, int WM, int WN, class FA, class FB, class EP>
inline void launch_gemm_x6(FA fa, FB fb, EP ep, int M, int N, int K, hipStream_t st) {
  if (M <= 0 || N <= 0) return;
  hipLaunchKernelGGL((gemm_x6_kernel<BM, BN, BK, WM, WN, FA, FB, EP>), grid_for(M, N, BM, BN), dim3(256), 0, st, fa, fb,
                     ep, M, N, K, K);
}

template <int BM, int BN, int BK, int WM, int WN, class FA, class FB, class EP>
inline void launch_gemm32(FA fa, FB fb, EP ep, int M, int N, int K, hipStream_t st, int splits = 1, int kchunk = 0) {
  if (M <= 0 || N <= 0) return;
  if (kchunk <= 0) kchunk = K;
  hipLaunchKernelGGL((gemm32_kernel<BM, BN, BK, WM, WN, FA, FB, EP>), grid_for(M, N, BM, BN, splits), dim3(256), 0,
                     st, fa, fb, ep, M, N, K, kchunk);
}

// Epilogue of a split-K product: element (row, col) = the fixed-order sum of its `splits`
// slab partials, then the product's own epilogue functor (any of its three forms).
// G > 1 (few outputs, many splits): G lanes per element, lane j summing splits z = j (mod G)
// in order, then a fixed xor tree (as wgrad_reduce_g_kernel).
template <class EP, int G = 1>
__global__ __launch_bounds__(256) void splitk_epilogue_kernel(const float* __restrict__ slab, int splits, int M, int N,
                                                              EP ep) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t idx = t / G;
  const int j = (int)(t - idx * G);
  const int64_t MN = (int64_t)M * N;
  float v = 0.0f;
  if (idx < MN)
    for (int z = j; z < splits; z += G) v += slab[z * MN + idx];
  if constexpr (G > 1) {
#pragma unroll
    for (int o = G / 2; o > 0; o >>= 1) v += __shfl_xor(v, o);
    if (j != 0) return;
  }
  if (idx >= MN) return;
  const int row = (int)(idx / N), col = (int)(idx - (idx / N) * N);
  if constexpr (has_pre_col<EP>::value)
    ep.post(row, col, v, ep.pre_col(col), 0);
  else if constexpr (has_pre_row<EP>::value)
    ep.post(row, col, v, ep.pre_row(row), 0);
  else if constexpr (has_pre<EP>::value)
    ep.post(row, col, v, ep.pre(row, col), 0);
  else
    ep(row, col, v, 0);
}

template <class EP>
inline void launch_splitk_epilogue(const float* slab, int splits, int M, int N, EP ep, hipStream_t st) {
  const int64_t MN = (int64_t)M * N;
  int G = 1;
  if (MN < 65536)
    while (G < 64 && G * 8 < splits) G *= 2;
  const unsigned blocks = (unsigned)((MN * G + 255) / 256);
  switch (G) {
    case 1: hipLaunchKernelGGL((splitk_epilogue_kernel<EP, 1>), dim3(blocks), dim3(256), 0, st, slab, splits, M, N, ep); break;
    case 2: hipLaunchKernelGGL((splitk_epilogue_kernel<EP, 2>), dim3(blocks), dim3(256), 0, st, slab, splits, M, N, ep); break;
    case 4: hipLaunchKernelGGL((splitk_epilogue_kernel<EP, 4>), dim3(blocks), dim3(256), 0, st, slab, splits, M, N, ep); break;
    case 8: hipLaunchKernelGGL((splitk_epilogue_kernel<EP, 8>), dim3(blocks), dim3(256), 0, st, slab, splits, M, N, ep); break;
    case 16: hipLaunchKernelGGL((splitk_epilogue_kernel<EP, 16>), dim3(blocks), dim3(256), 0, st, slab, splits, M, N, ep); break;
    case 32: hipLaunchKernelGGL((splitk_epilogue_kernel<EP, 32>), dim3(blocks), dim3(256), 0, st, slab, splits, M, N, ep); break;
    default: hipLaunchKernelGGL((splitk_epilogue_kernel<EP, 64>), dim3(blocks), dim3(256), 0, st, slab, splits, M, N, ep); break;
  }
}

// Splits of a product whose BM x BN tiles alone leave most of the chip idle (a 4-env rollout
// step: M = 4): the K range is cut into chunks of >= 2 K tiles so that ~512 workgroups run,
// partial products go to the policy's scratch slabs, and splitk_epilogue_kernel applies the
// epilogue. 1 = no split (every training batch of the bench: >= 128 tiles).
inline int splitk_count(int M, int N, int K, int BM, int BN, int BK, const PolicyLayout& L) {
  const int tiles = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  if (!L.sk || tiles >= 128 || K < 4 * BK) return 1;
  int dev = -1;
  if (hipGetDevice(&dev) != hipSuccess || dev != L.sk_dev) return 1;
  int splits = std::min((512 + tiles - 1) / tiles, K / (2 * BK));
  while (splits > 1 && (int64_t)splits * M * N > L.sk_cap) --splits;
  return std::max(splits, 1);
}

// BKN: the K tile of the unsplit form. 64 for conv_merge's forward and the LSTM's dh product
// (64 x 64 tiles, K 288-12512): the same MFMAs in the same k order as BK = 32 (bitwise equal
// output), half the barriers and twice the bytes per memory round trip (tools/gemm_x6_bench.hip
// mode 4: dh 75 -> 69 us, conv_merge at 174x174 89 -> 84 us per call); the split form keeps BK.
template <int BM, int BN, int BK, int WM, int WN, int BKN = BK, class FA, class FB, class EP>
inline void launch_gemm_x6_sk(FA fa, FB fb, EP ep, int M, int N, int K, hipStream_t st, const PolicyLayout& L) {
  if (M <= 0 || N <= 0) return;
  int splits = splitk_count(M, N, K, BM, BN, BK, L);
  if (splits <= 1) {
    launch_gemm_x6<BM, BN, BKN, WM, WN>(fa, fb, ep, M, N, K, st);
    return;
  }
  const int kchunk = ((K + splits - 1) / splits + BK - 1) / BK * BK;
  splits = (K + kchunk - 1) / kchunk;
  EpiSlab es{L.sk, M, N};
  hipLaunchKernelGGL((gemm_x6_kernel<BM, BN, BK, WM, WN, FA, FB, EpiSlab>), grid_for(M, N, BM, BN, splits), dim3(256),
                     0, st, fa, fb, es, M, N, K, kchunk);
  launch_splitk_epilogue(L.sk, splits, M, N, ep, st);
}

// The f32 MFMA core's form (the heads: N = actions + 1, K = 512).
template <int BM, int BN, int BK, int WM, int WN, class FA, class FB, class EP>
inline void launch_gemm_sk(FA fa, FB fb, EP ep, int M, int N, int K, hipStream_t st, const PolicyLayout& L) {
  if (M <= 0 || N <= 0) return;
  int splits = splitk_count(M, N, K, BM, BN, BK, L);
  if (splits <= 1) {
    launch_gemm<BM, BN, BK, WM, WN>(fa, fb, ep, M, N, K, st);
    return;
  }
  const int kchunk = ((K + splits - 1) / splits + BK - 1) / BK * BK;
  splits = (K + kchunk - 1) / kchunk;
  EpiSlab es{L.sk, M, N};
  launch_gemm<BM, BN, BK, WM, WN>(fa, fb, es, M, N, K, st, splits, kchunk);
  launch_splitk_epilogue(L.sk, splits, M, N, ep, st);
}

// Split-K wgrad: dW [M][KP] and db [M] of a layer from A^T (dZ [P][M]) x B (im2col [P][KP]).
template <int BM, int BN, int WM, int WN, class FB>
inline void launch_wgrad(const float* dZ, int64_t ldz, int M, FB fb, int KP, int P, float* slab, int64_t slab_cap,
                         float* dW, float* db, hipStream_t st) {
  constexpr int BK = 32;
  const int N = KP + (db ? 1 : 0);  // db == nullptr: no bias column
  const int tiles = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  int splits = std::max(1, std::min((2048 + tiles - 1) / tiles, (P + 255) / 256));
  while ((int64_t)splits * M * N > slab_cap && splits > 1) splits /= 2;
  int kchunk = (P + splits - 1) / splits;
  kchunk = (kchunk + BK - 1) / BK * BK;
  splits = (P + kchunk - 1) / kchunk;
  DenseT fa{dZ, ldz, M};
  if (splits == 1) {
    launch_gemm<BM, BN, BK, WM, WN>(fa, fb, EpiWgrad{dW, db, nullptr, KP}, M, N, P, st, 1, kchunk);
    return;
  }
  EpiSlab ep{slab, M, N};
  launch_gemm<BM, BN, BK, WM, WN>(fa, fb, ep, M, N, P, st, splits, kchunk);
  launch_wgrad_reduce(slab, splits, M, N, KP, dW, db, nullptr, st);
}

// The same split-K wgrad on the x6 core: both operands gathered along the reduction index
// (DenseT dZ, Im2colT im2col) and split into bf16 planes as they are staged.
template <int BM, int BN, int WM, int WN, class FB>
inline void launch_wgrad6(const float* dZ, int64_t ldz, int M, FB fb, int KP, int P, float* slab, int64_t slab_cap,
                          float* dW, float* db, hipStream_t st) {
  constexpr int BK = 32;
  const int N = KP + (db ? 1 : 0);  // db == nullptr: no bias column
  const int tiles = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  int splits = std::max(1, std::min((2048 + tiles - 1) / tiles, (P + 255) / 256));
  while ((int64_t)splits * M * N > slab_cap && splits > 1) splits /= 2;
  int kchunk = (P + splits - 1) / splits;
  kchunk = (kchunk + BK - 1) / BK * BK;
  splits = (P + kchunk - 1) / kchunk;
  DenseT fa{dZ, ldz, M};
  if (splits == 1) {
    hipLaunchKernelGGL((gemm_x6_kernel<BM, BN, BK, WM, WN, DenseT, FB, EpiWgrad>), grid_for(M, N, BM, BN, 1), dim3(256),
                       0, st, fa, fb, EpiWgrad{dW, db, nullptr, KP}, M, N, P, kchunk);
    return;
  }
  EpiSlab ep{slab, M, N};
  hipLaunchKernelGGL((gemm_x6_kernel<BM, BN, BK, WM, WN, DenseT, FB, EpiSlab>), grid_for(M, N, BM, BN, splits),
                     dim3(256), 0, st, fa, fb, ep, M, N, P, kchunk);
  launch_wgrad_reduce(slab, splits, M, N, KP, dW, db, nullptr, st);
}

// Split-K wgrad on the x6 core straight from the producers' [P][*] rows: dZ [P][ldz] as the
// transposed A (DenseT) and X [P][ldx] as the transposed B with the ones row (DenseTOnes), k =
// the P rows. The k-major staging (trans_slot_x6, frag_tr) hands the MFMAs the fragments the
// row-fill form reads from transposed copies, in the same k order: bitwise its output, without
// the two tile_transpose passes.
template <int BM, int BN, int WM, int WN>
inline void launch_wgrad_x6t(const float* dZ, int64_t ldz, int M, const float* X, int64_t ldx, int KP, int P,
                             float* slab, int64_t slab_cap, float* dW, float* db, hipStream_t st, float* db2 = nullptr) {
  constexpr int BK = 32;
  const int N = KP + (db ? 1 : 0);  // db == nullptr: no bias column
  const int tiles = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  int splits = std::max(1, std::min((2048 + tiles - 1) / tiles, (P + 255) / 256));
  while ((int64_t)splits * M * N > slab_cap && splits > 1) splits /= 2;
  int kchunk = (P + splits - 1) / splits;
  kchunk = (kchunk + BK - 1) / BK * BK;
  splits = (P + kchunk - 1) / kchunk;
  DenseT fa{dZ, ldz, M};
  DenseTOnes fb{X, ldx, KP};
  if (splits == 1) {
    hipLaunchKernelGGL((gemm_x6_kernel<BM, BN, BK, WM, WN, DenseT, DenseTOnes, EpiWgrad>), grid_for(M, N, BM, BN, 1),
                       dim3(256), 0, st, fa, fb, EpiWgrad{dW, db, db2, KP}, M, N, P, kchunk);
    return;
  }
  EpiSlab ep{slab, M, N};
  hipLaunchKernelGGL((gemm_x6_kernel<BM, BN, BK, WM, WN, DenseT, DenseTOnes, EpiSlab>), grid_for(M, N, BM, BN, splits),
                     dim3(256), 0, st, fa, fb, ep, M, N, P, kchunk);
  launch_wgrad_reduce(slab, splits, M, N, KP, dW, db, db2, st);
}

// Split-K wgrad on the x6 core from transposed operands: dZT [M][P] (rows = output
// channels, k = samples) and XT [KP][P] (+ the ones row), both row-fill. The producers'
// [P][*] tensors are transposed once (tile_transpose) so the reduction runs k-contiguous.
template <int BM, int BN, int WM, int WN>
inline void launch_wgrad_x6(const float* dZT, int M, const float* XT, int KP, int P, int64_t ldt, float* slab,
                            int64_t slab_cap, float* dW, float* db, hipStream_t st, float* db2 = nullptr) {
  constexpr int BK = 32;
  const int N = KP + (db ? 1 : 0);  // db == nullptr: no bias column
  const int tiles = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  int splits = std::max(1, std::min((2048 + tiles - 1) / tiles, (P + 255) / 256));
  while ((int64_t)splits * M * N > slab_cap && splits > 1) splits /= 2;
  int kchunk = (P + splits - 1) / splits;
  kchunk = (kchunk + BK - 1) / BK * BK;
  splits = (P + kchunk - 1) / kchunk;
  DenseRows fa{dZT, ldt, M};
  RowsOnes fb{XT, ldt, KP};
  EpiSlab ep{slab, M, N};
  hipLaunchKernelGGL((gemm_x6_kernel<BM, BN, BK, WM, WN, DenseRows, RowsOnes, EpiSlab>), grid_for(M, N, BM, BN, splits),
                     dim3(256), 0, st, fa, fb, ep, M, N, P, kchunk);
  launch_wgrad_reduce(slab, splits, M, N, KP, dW, db, db2, st);
}

// dgrad of one (group, parity) class of a k4 s2 conv: input pixels (y, x) with
// y % 2 == PY, x % 2 == PX of nimg images, masked by the ReLU of their producer.
template <int COUT, int CINF, int H, int W, int OH, int OW, int PY, int PX>
inline void dgrad_class(const float* dz, const float* WT, float* out, const float* X, int nimg, int g, int G, int cin,
                        hipStream_t st) {
  constexpr int HYC = (H - PY + 1) / 2, WXC = (W - PX + 1) / 2;
  const int M = nimg * HYC * WXC;
  DgradA<COUT, 4, 2, OH, OW, HYC, WXC> fa{dz, M};
  DgradB<COUT, 4, 2, CINF> fb{WT, cin, g * cin, PY, PX};
  EpiMaskParity<H, W, 2, PY, PX, HYC, WXC> ep{out, X, g, G, cin};
  launch_gemm_x6<128, 32, 32, 4, 1>(fa, fb, ep, M, cin, 4 * COUT, st);
}

// All G input-channel groups of a class in one product (N = G * cin): the gathered and
// split dZ operand serves twice the columns.
// Rows / columns of an H x W input that a k4 s2 conv with an OH x OW output reads at all
// (84x84 conv3: 8 of 9 — row 8 and column 8 get no gradient).
template <int H, int OH>
constexpr int k4s2_covered() {
  return H < 2 * (OH - 1) + 4 ? H : 2 * (OH - 1) + 4;
}

// dX = 0 at the input pixels no output window covers (all G groups of every image).
template <int H, int W, int CH, int CW>
__global__ void zero_uncovered_kernel(float* __restrict__ out, int nimg_g, int cin) {
  constexpr int NU = H * W - CH * CW;  // uncovered pixels per image
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int c4n = cin / 4;
  if (i >= (int64_t)nimg_g * NU * c4n) return;
  const int c4 = (int)(i % c4n);
  const int64_t q = i / c4n;
  const int u = (int)(q % NU);
  const int64_t ng = q / NU;
  int y, x;
  if (u < (H - CH) * W) {  // whole uncovered rows
    y = CH + u / W;
    x = u % W;
  } else {  // uncovered columns of the covered rows
    const int v = u - (H - CH) * W;
    y = v / (W - CW);
    x = CW + v % (W - CW);
  }
  *reinterpret_cast<f4*>(out + ((ng * H + y) * W + x) * cin + 4 * c4) = f4zero();
}

// Stride-2 k4 parity-class products on bf16 MFMA with split operands, all four classes
// (py, px) in one persistent kernel: output pixel (2yy + py, 2xx + px) sums, over the 2x2
// taps (ky, kx) = (py + 2 tky, px + 2 tkx) that reach it, the staged map's pixel
// (yy - tky, xx - tkx) (KC channels) times W[tap][col][KC]. Two products use it: conv3's input
// gradient (map dZ3, 64 -> 2 x 32 channels under X2's ReLU) and the aux heads' first
// transposed conv (map X4, 32 -> 48 channels, bias + ReLU) — the x6 scheme of
// conv2_dgrad_x6_kernel (vn_conv1.h). Wave w owns class w / WPC and the NTL 16-wide column
// tiles of column group w % WPC; its split weights (4 taps x KC/32 k steps x NTL tiles x 3
// terms) stay in registers for the kernel's lifetime. A work item is IMG images: their maps
// are split once when staged (three bf16 planes), where the generic class products re-split
// every map value at each of its 16 uses (22 VALU per MFMA). Plane rows as in
// conv2_dgrad_x6_kernel: map pixel (oy, ox) of item image im at row im NPC + (oy + 1) XC +
// ox + 1 (XC = SW + 1, YC = SH + 1: an image's rows, padding included, are exactly its NPC
// class pixels), so every tap of a 16-pixel tile reads 16 consecutive rows; out-of-range taps
// read rows no pixel owns (zeroed once); quads rotated per row (dg_quad_off): no bank
// conflicts on the fragment reads (the former KC + 8 padded rows with a shared zero row
// conflicted 2-way, 0.55 of the LDS cycles). The product is transposed (rows = columns of W, MFMA columns = class pixels), so
// each lane hands the epilogue 4 consecutive channels of one output pixel.
template <int SH_, int SW_, int YC_, int XC_, int KC_, int NCOL_, int WPC_>
struct ParityDg {
  static constexpr int SH = SH_, SW = SW_, YC = YC_, XC = XC_, KC = KC_, NCOL = NCOL_, WPC = WPC_;
  static constexpr int NP = SH * SW;                     // staged map pixels per image
  static constexpr int NPC = YC * XC;                    // class pixels per image
  static constexpr int PS = KC + 8;                      // banded form's plane row stride (bf16)
  static constexpr int rows(int img) { return (img * NPC + 15) / 16 * 16 + XC + 1; }  // + the last tile's reads
  // images per work item: >= 64 class pixels; two large maps where their planes fit (the
  // next item then loads at the item's start: prefetch registers would spill), one else
  static constexpr int IMG = NPC >= 64 ? ((size_t)3 * rows(2) * KC * 2 <= 160 * 1024 ? 2 : 1) : 64 / NPC;
  static constexpr int NR = rows(IMG);
  static constexpr int NTL = NCOL / (16 * WPC);          // column tiles per wave
  static constexpr int KS = KC / 32;                     // MFMA k steps per tap
  static constexpr int NT = 256 * WPC;
  static constexpr size_t LDS = (size_t)3 * NR * KC * 2;
  static constexpr bool fits = LDS <= 160 * 1024;
  static_assert(KC % 32 == 0 && NCOL % (16 * WPC) == 0, "k steps of 32, whole 16-column tiles per wave");
  static_assert(KC == 32 || KC == 64, "plane rows of 4 or 8 quads (dg_quad_off)");
  static_assert(XC == SW + 1 && YC == SH + 1, "k4 s2 classes: the map plus one gap row and column");
};

template <class S, class EP>
__global__ __launch_bounds__(S::NT, S::NT >= 512 ? 1 : 2) void parity_dgrad_x6_kernel(const float* __restrict__ map,
                                                                const float* __restrict__ WT, EP ep, int n) {
  constexpr int SW = S::SW, XC = S::XC, KC = S::KC, NCOL = S::NCOL, WPC = S::WPC;
  constexpr int NP = S::NP, NPC = S::NPC, IMG = S::IMG, NTL = S::NTL, KS = S::KS, NT = S::NT;
  constexpr int ROWS = IMG * NP, PL = S::NR * KC, C4 = KC / 4, NQ = KC / 8;
  constexpr int TILES = (IMG * NPC + 15) / 16, NZ = (ROWS * C4 + NT - 1) / NT;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem_pdg[];
  uint16_t* zs = reinterpret_cast<uint16_t*>(smem_pdg);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int cls = wave / WPC, py = cls >> 1, px = cls & 1;
  const int col0 = (wave % WPC) * NTL * 16;
  const int i16 = lane & 15, q = lane >> 4;
  bf16x8_t bw[4][KS][NTL][3];  // [tap][k step][column tile][term]: A[col][k = 32h + 8q + j]
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int ky = py + 2 * (t >> 1), kx = px + 2 * (t & 1);
#pragma unroll
    for (int h = 0; h < KS; ++h)
#pragma unroll
      for (int nt = 0; nt < NTL; ++nt) {
        union { uint16_t u[8]; bf16x8_t v; } b0, b1, b2;
        const float* w = WT + ((int64_t)(ky * 4 + kx) * NCOL + col0 + 16 * nt + i16) * KC + 32 * h + 8 * q;
#pragma unroll
        for (int j = 0; j < 8; ++j) split3_bf16(w[j], b0.u[j], b1.u[j], b2.u[j]);
        bw[t][h][nt][0] = b0.v;
        bw[t][h][nt][1] = b1.v;
        bw[t][h][nt][2] = b2.v;
      }
  }
  // every plane row zero once (rows no map pixel owns stay zero); the barrier orders these
  // stores before the first item's
  for (int i = tid; i < 3 * PL / 8; i += NT) reinterpret_cast<uint4*>(zs)[i] = uint4{0u, 0u, 0u, 0u};
  __syncthreads();
  const int items = (n + IMG - 1) / IMG;
  f4 zr[NZ];
  auto load_z = [&](int it) {  // the item's map rows (images consecutive), zeros past n
    const int64_t r0 = (int64_t)it * ROWS, rend = (int64_t)n * NP;
    const f4* z4 = reinterpret_cast<const f4*>(map);
#pragma unroll
    for (int j = 0; j < NZ; ++j) {
      const int i = tid + j * NT;
      if (i < ROWS * C4) zr[j] = r0 + i / C4 < rend ? z4[(r0 + i / C4) * C4 + i % C4] : f4zero();
    }
  };
  // the next item's map is prefetched into registers while this one multiplies, unless it
  // would not fit beside the weights (two 9x9 maps, 300x400's 17x23 map: loaded at the
  // item's start)
  constexpr bool PF = NZ <= 3;
  if (PF && (int)blockIdx.x < items) load_z(blockIdx.x);
  for (int it = blockIdx.x; it < items; it += gridDim.x) {
    if constexpr (!PF) load_z(it);
#pragma unroll
    for (int j = 0; j < NZ; ++j) {
      const int i = tid + j * NT;
      if (i < ROWS * C4) {
        uint2 t0, t1, t2;
        split3_pack(zr[j], t0, t1, t2);
        const int pix = i / C4, c = i - (i / C4) * C4, im = pix / NP, rem = pix - (pix / NP) * NP;
        const int row = im * NPC + (rem / SW + 1) * XC + rem % SW + 1;
        uint16_t* d = zs + dg_quad_off<NQ>(row, c >> 1) + 4 * (c & 1);
        *reinterpret_cast<uint2*>(d) = t0;
        *reinterpret_cast<uint2*>(d + PL) = t1;
        *reinterpret_cast<uint2*>(d + 2 * PL) = t2;
      }
    }
    __syncthreads();
    if (PF && it + (int)gridDim.x < items) load_z(it + gridDim.x);
    const int img0 = it * IMG;
#pragma unroll 1
    for (int tile = 0; tile < TILES; ++tile) {
      const int pc = tile * 16 + i16;  // this lane's class pixel (MFMA column) within the item
      const int im = pc / NPC, r = pc - (pc / NPC) * NPC;
      const int yy = r / XC, xx = r - (r / XC) * XC;
      const bool live = pc < IMG * NPC && img0 + im < n;
      int row[4];  // tap (ty, tx) reads row pc + (1 - ty) XC + (1 - tx)
#pragma unroll
      for (int tap = 0; tap < 4; ++tap) row[tap] = pc + (1 - (tap >> 1)) * XC + (1 - (tap & 1));
      f4 acc[NTL];
#pragma unroll
      for (int nt = 0; nt < NTL; ++nt) acc[nt] = f4zero();
#pragma unroll
      for (int tap = 0; tap < 4; ++tap)
#pragma unroll
        for (int h = 0; h < KS; ++h) {
          bf16x8_t a[3];
#pragma unroll
          for (int tm = 0; tm < 3; ++tm)
            a[tm] = *reinterpret_cast<const bf16x8_t*>(zs + tm * PL + dg_quad_off<NQ>(row[tap], q + 4 * h));
#pragma unroll
          for (int nt = 0; nt < NTL; ++nt) {  // small terms first
            f4 c = acc[nt];
            c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bw[tap][h][nt][0], a[2], c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bw[tap][h][nt][2], a[0], c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bw[tap][h][nt][1], a[1], c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bw[tap][h][nt][0], a[1], c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bw[tap][h][nt][1], a[0], c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bw[tap][h][nt][0], a[0], c, 0, 0, 0);
            acc[nt] = c;
          }
        }
      if (live) {  // lane (pixel, q) holds columns col0 + 16 nt + 4q .. +3
        // every epilogue load before the first store: vmcnt counts stores too, so a load
        // issued after a store would wait for it (+8 % per launch measured)
        const int y = 2 * yy + py, x = 2 * xx + px;
        f4 pre[NTL];
#pragma unroll
        for (int nt = 0; nt < NTL; ++nt) pre[nt] = ep.pre(img0 + im, y, x, col0 + 16 * nt + 4 * q);
#pragma unroll
        for (int nt = 0; nt < NTL; ++nt) ep.post(img0 + im, y, x, col0 + 16 * nt + 4 * q, acc[nt], pre[nt]);
      }
    }
    __syncthreads();
  }
}

// The same product for maps whose planes do not fit whole (300x400: the 17x23x64 dZ3 map is 169
// KB of planes): work item = (image, band of BY class rows yy), staging the BY + 1 map rows its
// taps read (rows yy - 1 .. yy + BY - 1, staged as zeros outside the map). Plane rows as in the
// whole-map form: staged row j, pixel ox at row j XC + ox + 1, so band pixel pc = yl XC + xx
// reads row pc + (1 - ty) XC + (1 - tx); column 0 is never written (zero); quads rotated. Same
// fragments and MFMA order per output (bit-identical to the whole-map form).
template <class S, int BY>
constexpr int parity_band_nr() {  // plane rows: the last tile's reads
  return (BY * S::XC + 15) / 16 * 16 + S::XC + 1;
}
template <class S, int BY>
constexpr size_t parity_band_lds() {
  return (size_t)3 * parity_band_nr<S, BY>() * S::KC * 2;
}

template <class S, int BY, class EP>
__global__ __launch_bounds__(S::NT, 1) void parity_dgrad_band_x6_kernel(const float* __restrict__ map,
                                                                       const float* __restrict__ WT, EP ep, int n) {
  constexpr int SH = S::SH, SW = S::SW, YC = S::YC, XC = S::XC, KC = S::KC, NCOL = S::NCOL, WPC = S::WPC;
  constexpr int NTL = S::NTL, KS = S::KS, NT = S::NT, NQ = KC / 8;
  constexpr int NB = (YC + BY - 1) / BY;                       // bands per image
  constexpr int ROWS = (BY + 1) * SW, PL = parity_band_nr<S, BY>() * KC, C4 = KC / 4;
  constexpr int TILES = (BY * XC + 15) / 16, NZ = (ROWS * C4 + NT - 1) / NT;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem_pdb[];
  uint16_t* zs = reinterpret_cast<uint16_t*>(smem_pdb);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int cls = wave / WPC, py = cls >> 1, px = cls & 1;
  const int col0 = (wave % WPC) * NTL * 16;
  const int i16 = lane & 15, q = lane >> 4;
  bf16x8_t bw[4][KS][NTL][3];
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int ky = py + 2 * (t >> 1), kx = px + 2 * (t & 1);
#pragma unroll
    for (int h = 0; h < KS; ++h)
#pragma unroll
      for (int nt = 0; nt < NTL; ++nt) {
        union { uint16_t u[8]; bf16x8_t v; } b0, b1, b2;
        const float* w = WT + ((int64_t)(ky * 4 + kx) * NCOL + col0 + 16 * nt + i16) * KC + 32 * h + 8 * q;
#pragma unroll
        for (int j = 0; j < 8; ++j) split3_bf16(w[j], b0.u[j], b1.u[j], b2.u[j]);
        bw[t][h][nt][0] = b0.v;
        bw[t][h][nt][1] = b1.v;
        bw[t][h][nt][2] = b2.v;
      }
  }
  // every plane row zero once (column 0 of the staged rows stays zero); the barrier orders
  // these stores before the first item's
  for (int i = tid; i < 3 * PL / 8; i += NT) reinterpret_cast<uint4*>(zs)[i] = uint4{0u, 0u, 0u, 0u};
  __syncthreads();
  const int items = n * NB;
  for (int it = blockIdx.x; it < items; it += gridDim.x) {
    const int img = it / NB, y0 = (it - (it / NB) * NB) * BY;
    {  // map rows y0 - 1 .. y0 + BY - 1 of the image (rows outside the map stage zeros)
      const f4* z4 = reinterpret_cast<const f4*>(map) + (int64_t)img * SH * SW * C4;
#pragma unroll 2
      for (int j = 0; j < NZ; ++j) {
        const int i = tid + j * NT;
        if (i < ROWS * C4) {
          const int rp = i / C4, c = i - (i / C4) * C4;
          const int oy = y0 - 1 + rp / SW;
          const f4 v = (oy >= 0 && oy < SH) ? z4[((int64_t)oy * SW + rp % SW) * C4 + c] : f4zero();
          uint2 t0, t1, t2;
          split3_pack(v, t0, t1, t2);
          uint16_t* d = zs + dg_quad_off<NQ>((rp / SW) * XC + rp % SW + 1, c >> 1) + 4 * (c & 1);
          *reinterpret_cast<uint2*>(d) = t0;
          *reinterpret_cast<uint2*>(d + PL) = t1;
          *reinterpret_cast<uint2*>(d + 2 * PL) = t2;
        }
      }
    }
    __syncthreads();
#pragma unroll 1
    for (int tile = 0; tile < TILES; ++tile) {
      const int pc = tile * 16 + i16;  // this lane's class pixel (MFMA column) within the band
      const int yl = pc / XC, xx = pc - (pc / XC) * XC, yy = y0 + yl;
      const bool live = pc < BY * XC && yy < YC;
      int row[4];  // tap (ty, tx) reads row pc + (1 - ty) XC + (1 - tx)
#pragma unroll
      for (int tap = 0; tap < 4; ++tap) row[tap] = pc + (1 - (tap >> 1)) * XC + (1 - (tap & 1));
      f4 acc[NTL];
#pragma unroll
      for (int nt = 0; nt < NTL; ++nt) acc[nt] = f4zero();
#pragma unroll
      for (int tap = 0; tap < 4; ++tap)
#pragma unroll
        for (int h = 0; h < KS; ++h) {
          bf16x8_t a[3];
#pragma unroll
          for (int tm = 0; tm < 3; ++tm)
            a[tm] = *reinterpret_cast<const bf16x8_t*>(zs + tm * PL + dg_quad_off<NQ>(row[tap], q + 4 * h));
#pragma unroll
          for (int nt = 0; nt < NTL; ++nt) {  // small terms first
            f4 c = acc[nt];
            c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bw[tap][h][nt][0], a[2], c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bw[tap][h][nt][2], a[0], c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bw[tap][h][nt][1], a[1], c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bw[tap][h][nt][0], a[1], c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bw[tap][h][nt][1], a[0], c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bw[tap][h][nt][0], a[0], c, 0, 0, 0);
            acc[nt] = c;
          }
        }
      if (live) {
        const int y = 2 * yy + py, x = 2 * xx + px;
        f4 pre[NTL];
#pragma unroll
        for (int nt = 0; nt < NTL; ++nt) pre[nt] = ep.pre(img, y, x, col0 + 16 * nt + 4 * q);
#pragma unroll
        for (int nt = 0; nt < NTL; ++nt) ep.post(img, y, x, col0 + 16 * nt + 4 * q, acc[nt], pre[nt]);
      }
    }
    __syncthreads();
  }
}

// class rows per band of the banded parity product: the bands the largest that fits 150 KB
// needs, evened out (300x400: 18 class rows -> 2 bands of 9)
template <class S>
constexpr int parity_band_rows() {
  int bmax = 0;
  for (int b = S::YC; b >= 1 && bmax == 0; --b)
    if ((size_t)3 * ((b * S::XC + 15) / 16 * 16 + S::XC + 1) * S::KC * 2 <= 150 * 1024) bmax = b;
  if (bmax == 0) return 0;
  const int nb = (S::YC + bmax - 1) / bmax;
  return (S::YC + nb - 1) / nb;
}

// conv3's input gradient: column c is channel c % 32 of input group c / 32 (X2 layout
// [n][2][IH][IW][32]), masked by the ReLU that produced X2 (as EpiMaskParityG).
// mask_goal == 0 (goal-frame deduplication): group 1 is left unmasked — a sample's goal map
// lives at its run start, where goal_dz2_reduce_kernel sums the run and applies the mask.
template <int IH, int IW>
struct EpiDgMaskG2 {
  const float* X;
  float* out;
  int mask_goal = 1;
  __device__ __forceinline__ int64_t index(int img, int y, int x, int col) const {
    return ((((int64_t)img * 2 + (col >> 5)) * IH + y) * IW + x) * 32 + (col & 31);
  }
  __device__ __forceinline__ f4 pre(int img, int y, int x, int col) const {
    return *reinterpret_cast<const f4*>(X + index(img, y, x, col));
  }
  __device__ __forceinline__ void post(int img, int y, int x, int col, f4 v, f4 xm) const {
    const bool m = mask_goal || col < 32;
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = (!m || xm[e] > 0.0f) ? v[e] : 0.0f;
    *reinterpret_cast<f4*>(out + index(img, y, x, col)) = v;
  }
};

// Goal-frame deduplication, backward: the goal map gradient of a run = the sum of its
// samples' (conv3's unmasked input gradient, group 1) in step order, under the ReLU of the
// run's goal map: dZ2[2r+1] = [X2[2r+1] > 0] * sum_{i < len} dX2[2(r + iE) + 1] for every run
// start r. One thread per (run, channel quad of a pixel); the run count is on the device.
__global__ __launch_bounds__(256) void goal_dz2_reduce_kernel(float* __restrict__ dz2, const float* __restrict__ X2,
                                                              int64_t frame_f4, const int32_t* __restrict__ list,
                                                              const int32_t* __restrict__ count,
                                                              const int32_t* __restrict__ run_length, int E) {
  const int64_t total = (int64_t)(*count) * frame_f4;
  for (int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x; idx < total; idx += (int64_t)gridDim.x * 256) {
    const int64_t j = idx / frame_f4, c = idx - j * frame_f4;
    const int64_t r = list[j];
    const int len = run_length[r];
    f4* d = reinterpret_cast<f4*>(dz2) + (2 * r + 1) * frame_f4 + c;
    f4 acc = *d;
    for (int i = 1; i < len; ++i) acc += reinterpret_cast<const f4*>(dz2)[(2 * (r + (int64_t)i * E) + 1) * frame_f4 + c];
    const f4 x = reinterpret_cast<const f4*>(X2)[(2 * r + 1) * frame_f4 + c];
#pragma unroll
    for (int e = 0; e < 4; ++e) acc[e] = x[e] > 0.0f ? acc[e] : 0.0f;
    *d = acc;
  }
}

// Transposed conv output: bias (+ ReLU), NHWC with C channels (as EpiDeconv).
template <int OH, int OW, int C>
struct EpiDgBias {
  float* out;
  const float* bias;
  int relu;
  __device__ __forceinline__ f4 pre(int, int, int, int col) const {
    return *reinterpret_cast<const f4*>(bias + col);
  }
  __device__ __forceinline__ void post(int img, int y, int x, int col, f4 v, f4 b) const {
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = relu ? fmaxf(v[e] + b[e], 0.0f) : v[e] + b[e];
    *reinterpret_cast<f4*>(out + (((int64_t)img * OH + y) * OW + x) * C + col) = v;
  }
};

template <class S, class EP>
inline int launch_parity_dgrad_x6(const float* map, const float* WT, EP ep, int n, hipStream_t st) {
  const void* kfn = (const void*)parity_dgrad_x6_kernel<S, EP>;
  VN_HIP(ensure_dyn_lds(kfn, S::LDS));
  const int items = (n + S::IMG - 1) / S::IMG;
  const int blocks = std::min(items, resident_blocks(kfn, S::NT, S::LDS));
  if (blocks > 0) hipLaunchKernelGGL((parity_dgrad_x6_kernel<S, EP>), dim3(blocks), dim3(S::NT), S::LDS, st, map, WT, ep, n);
  return VN_OK;
}

// Weight gradient of a k4 s2 conv with 32-channel input groups on bf16 MFMA with split
// operands: dW[co][tap][g, ci] = sum over images and dZ pixels o of dZ[o][co] *
// X[g][2oy + ky][2ox + kx][ci], db[co] = sum of dZ[o][co] — conv3 (64 <- 2 x 32 channels)
// and conv2 (32 <- 32, image and goal frames as separate images). The generic split-K
// product gathered each X value once per tap (4x) and split it at every use; conv2's f32
// kernel ran its pipe at 85 %. Here a workgroup (input group g = blockIdx.y) stages a work
// item — IMG images x a band of BR dZ rows, with the 2 BR + 2 X rows under it — split once
// into bf16 LDS planes in their natural [pixel][channel] layout, and reads both MFMA operands
// with ds_read_b64_tr_b16, whose per-lane row addresses do the im2col gather for free: the
// reduction index k runs over the item's dZ pixels (32 per 16x16x32 step), so the A fragment
// (co x 8 pixels) reads dZ rows k and the B fragment ((tap, ci) x 8 pixels) reads the X rows
// under each pixel's tap. Wave w owns taps 2w, 2w+1: CO/16 co tiles x 4 (tap, ci) tiles of
// accumulators, kept across all of the workgroup's items; each workgroup writes one partial
// slab row, reduced in a fixed order by wgrad_reduce_kernel (the bias from the g = 0
// workgroups' fp32 column sums of dZ). The next item is prefetched into registers.
template <int IH_, int IW_, int OH_, int OW_, int CO_, int G_, int BR_, int IMG_, int CX_ = 32, bool BIAS_ = true>
struct WgSpec {
  static constexpr int IH = IH_, IW = IW_, OH = OH_, OW = OW_, CO = CO_, G = G_, BR = BR_, IMG = IMG_;
  static constexpr int CX = CX_;        // X channels per input group (32, or the aux heads' 48)
  static constexpr bool BIAS = BIAS_;   // a bias column (the aux heads take theirs from column sums)
  static constexpr int NTW = CX / 16;   // (tap, channel) tiles per tap
  static constexpr int NB = OH / BR;                        // bands per image
  static constexpr int XR = 2 * BR + 2 < IH ? 2 * BR + 2 : IH;  // X rows under a band
  static constexpr int NPX = XR * IW;                       // staged X pixels per image
  static constexpr int KP = IMG * BR * OW, KSTEPS = (KP + 31) / 32;
  // k order and plane row strides (bf16): with KPERM the 8 rows a 32-lane half of a
  // transpose read touches (pixels k..k+7) start 8-bank multiples apart on distinct banks —
  // dZ rows PZ/2 banks apart (PZ = 48 / 80), X rows 2 pixels = PX banks apart (PX = 40). The
  // aux heads' 48-channel form keeps the plain order (the permuted one spilled there).
  static constexpr bool KPERM = CX == 32;
  static constexpr int PZ = CO + (KPERM ? 16 : 8), PX = CX + 8;
  static constexpr int RZ = KP + 1, RX = IMG * NPX + 1;     // rows + one zero row each
  static constexpr size_t LDS = (size_t)3 * (RZ * PZ + RX * PX) * 2;
  static constexpr bool fits = OH % BR == 0 && LDS <= 160 * 1024;
  static constexpr int KW = 16 * G * CX;                     // weight columns
  static constexpr int SLAB_N = KW + (BIAS ? 1 : 0);          // + the bias
  static constexpr int MT = CO / 16, C4 = CO / 4;
};

__device__ __forceinline__ s16x4_ lds_tr(const uint16_t* p) {
  typedef __attribute__((address_space(3))) s16x4_ lds_s16x4;
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p));
}

// Staging slot i -> (row, 4-channel chunk) of a plane with Q chunks a row and a row stride of
// RSTRIDE dwords: with Q = 8 the 16 lanes of a ds_write_b64 group take rows r and r + D, D
// chosen so that D RSTRIDE = 16 mod 32 (their 16-dword runs on disjoint banks; rows r, r + 1
// overlapped 2-way at strides 20 and 24), in whole blocks of 2D rows; the tail rows and other
// widths keep the identity. Loads and stores share it (tools/wgrad_banks.py).
template <int Q, int RSTRIDE, int ROWS>
__device__ __forceinline__ void wg_slot(int i, int& row, int& c) {
  constexpr int D = (Q == 8 && RSTRIDE % 32 == 20) ? 4 : (Q == 8 && RSTRIDE % 32 == 24) ? 2 : 0;
  c = i % Q;
  const int t = i / Q;
  if constexpr (D > 0) {
    constexpr int FULL = ROWS / (2 * D) * (2 * D);
    const int m = t % (2 * D);
    row = t < FULL ? t - m + (m >> 1) + (m & 1) * D : t;
  } else {
    row = t;
  }
}

template <class S>
// fl: the images (frames) to reduce over (conv2 with goal-frame deduplication; identity
// else). gdelta (conv3 with deduplication): input group 1 (the goal half of X2) of sample s is
// read from sample s + gdelta[s], the sample whose goal frame holds its goal's map.
__global__ __launch_bounds__(512, 1) void conv_wgrad_x6_kernel(const float* __restrict__ dZ, const float* __restrict__ X,
                                                            float* __restrict__ slab, int n, FrameList fl,
                                                            const int32_t* __restrict__ gdelta) {
  constexpr int IH = S::IH, IW = S::IW, OH = S::OH, OW = S::OW, CO = S::CO, G = S::G, BR = S::BR, IMG = S::IMG;
  constexpr int NPX = S::NPX, KP = S::KP, PZ = S::PZ, PX = S::PX, MT = S::MT, C4 = S::C4;
  constexpr int CX = S::CX, X4 = CX / 4, NTW = S::NTW, NTT = 2 * NTW;
  constexpr int PLZ = S::RZ * PZ, PLX = S::RX * PX, NT = 512, BP = BR * OW;
  constexpr int NZ = (KP * C4 + NT - 1) / NT, NX = (IMG * NPX * X4 + NT - 1) / NT;
  static_assert(NT % C4 == 0, "a thread's dZ channel quad is fixed");
  extern __shared__ __attribute__((aligned(16))) uint8_t smem_wg[];
  uint16_t* zs = reinterpret_cast<uint16_t*>(smem_wg);
  uint16_t* xs = zs + 3 * PLZ;
  float* red = reinterpret_cast<float*>(smem_wg);  // bias reduction, after the last item
  const int g = blockIdx.y;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int Gq = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  for (int i = tid; i < 3 * (PZ + PX) / 2; i += NT) {  // zero rows
    const int pl = i / ((PZ + PX) / 2), e = i - pl * ((PZ + PX) / 2);
    if (e < PZ / 2)
      reinterpret_cast<uint32_t*>(zs + pl * PLZ + KP * PZ)[e] = 0u;
    else
      reinterpret_cast<uint32_t*>(xs + pl * PLX + IMG * NPX * PX)[e - PZ / 2] = 0u;
  }
  f4 acc[MT][NTT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int nt = 0; nt < NTT; ++nt) acc[mt][nt] = f4zero();
  f4 dbs = f4zero();  // fp32 column sums of dZ (channels 4 (tid % C4) .. +3), g == 0 only
  n = fl_count(fl, n);
  const int items = (n + IMG - 1) / IMG * S::NB;
  f4 zr[NZ], xr[NX];
  // the item's dZ band rows and the X rows under them, into registers: unconditional (a slot
  // past the item or an image past n reloads a valid one; the split zeroes it), so no branch
  // hides the loads from the compiler's wait counts. The item's image indices (list entries,
  // goal redirection) are resolved first with scalar loads.
  auto load = [&](int it) {
    const int img0 = (it / S::NB) * IMG, band = it - (it / S::NB) * S::NB;
    int zi[IMG], xi[IMG];
#pragma unroll
    for (int im = 0; im < IMG; ++im) {
      zi[im] = fl_frame(fl, min(img0 + im, n - 1));
      xi[im] = zi[im] + ((gdelta && g == 1) ? fl_sload(gdelta + zi[im]) : 0);
    }
#pragma unroll
    for (int j = 0; j < NZ; ++j) {
      int k, c;
      wg_slot<C4, PZ / 2, KP>(min(tid + j * NT, KP * C4 - 1), k, c);
      const int im = k / BP;
      int imc = zi[0];  // select chain over the item's images (registers, no indexed array)
#pragma unroll
      for (int m = 1; m < IMG; ++m) imc = im == m ? zi[m] : imc;
      zr[j] = reinterpret_cast<const f4*>(dZ)[(((int64_t)imc * OH + band * BR) * OW + (k - im * BP)) * C4 + c];
    }
#pragma unroll
    for (int j = 0; j < NX; ++j) {
      int r, c;
      wg_slot<X4, PX / 2, IMG * NPX>(min(tid + j * NT, IMG * NPX * X4 - 1), r, c);
      const int im = r / NPX;
      int imc = xi[0];
#pragma unroll
      for (int m = 1; m < IMG; ++m) imc = im == m ? xi[m] : imc;
      xr[j] = reinterpret_cast<const f4*>(X)[((((int64_t)imc * G + g) * IH + 2 * band * BR) * IW + (r - im * NPX)) * X4 + c];
    }
  };
  if ((int)blockIdx.x < items) load(blockIdx.x);
  for (int it = blockIdx.x; it < items; it += gridDim.x) {
    const int img0 = (it / S::NB) * IMG;
#pragma unroll
    for (int j = 0; j < NZ; ++j) {  // split into the planes
      const int i = tid + j * NT;
      if (i < KP * C4) {
        int k, c;
        wg_slot<C4, PZ / 2, KP>(i, k, c);
        const f4 z = img0 + k / BP < n ? zr[j] : f4zero();
        if (S::BIAS && g == 0) dbs += z;
        uint2 t0, t1, t2;
        split3_pack(z, t0, t1, t2);
        uint16_t* d = zs + k * PZ + 4 * c;
        *reinterpret_cast<uint2*>(d) = t0;
        *reinterpret_cast<uint2*>(d + PLZ) = t1;
        *reinterpret_cast<uint2*>(d + 2 * PLZ) = t2;
      }
    }
#pragma unroll
    for (int j = 0; j < NX; ++j) {
      const int i = tid + j * NT;
      if (i < IMG * NPX * X4) {
        int r, c;
        wg_slot<X4, PX / 2, IMG * NPX>(i, r, c);
        const f4 x = img0 + r / NPX < n ? xr[j] : f4zero();
        uint2 t0, t1, t2;
        split3_pack(x, t0, t1, t2);
        uint16_t* d = xs + r * PX + 4 * c;
        *reinterpret_cast<uint2*>(d) = t0;
        *reinterpret_cast<uint2*>(d + PLX) = t1;
        *reinterpret_cast<uint2*>(d + 2 * PLX) = t2;
      }
    }
    __syncthreads();
    load(min(it + (int)gridDim.x, items - 1));  // next item's loads under this one's MFMAs
    auto kstep = [&](int ks) {
      // this lane's rows of the two tr reads: with KPERM the MFMA's k slot 8 Gq + 4s + q takes
      // item pixel 32 ks + 16 (Gq >> 1) + 8s + 4 (Gq & 1) + q (any bijection works when A and B
      // share it; this one puts a 32-lane half's two lane groups on 8 consecutive pixels per
      // read): dZ row k and, per tap
      // of the wave, the X row under it (the zero rows past the item)
      int zrow[2], xrow[2][2];
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int k = S::KPERM ? ks * 32 + 16 * (Gq >> 1) + 8 * s + 4 * (Gq & 1) + q : ks * 32 + 8 * Gq + 4 * s + q;
        const int im = k / BP, o = k - (k / BP) * BP;
        const int oy = o / OW, ox = o - (o / OW) * OW;  // oy within the band
        const bool ok = k < KP;
        zrow[s] = (ok ? k : KP) * PZ;
#pragma unroll
        for (int tt = 0; tt < 2; ++tt) {
          const int tap = 2 * wave + tt, ky = tap >> 2, kx = tap & 3;
          xrow[s][tt] = (ok ? im * NPX + (2 * oy + ky) * IW + 2 * ox + kx : IMG * NPX) * PX;
        }
      }
      bf16x8_ a[3][MT], b[3][NTT];
      union U { s16x4_ s[2]; bf16x8_ v; };
#pragma unroll
      for (int t = 0; t < 3; ++t) {
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {  // A: co 16 mt + (lane & 15) x pixels
          U u;
          u.s[0] = lds_tr(zs + t * PLZ + zrow[0] + 16 * mt + 4 * p);
          u.s[1] = lds_tr(zs + t * PLZ + zrow[1] + 16 * mt + 4 * p);
          a[t][mt] = u.v;
        }
#pragma unroll
        for (int nt = 0; nt < NTT; ++nt) {  // B: (tap 2w + nt / NTW, channel 16 (nt % NTW) + (lane & 15)) x pixels
          U u;
          u.s[0] = lds_tr(xs + t * PLX + xrow[0][nt / NTW] + 16 * (nt % NTW) + 4 * p);
          u.s[1] = lds_tr(xs + t * PLX + xrow[1][nt / NTW] + 16 * (nt % NTW) + 4 * p);
          b[t][nt] = u.v;
        }
      }
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int nt = 0; nt < NTT; ++nt) {  // small terms first
          f4 c = acc[mt][nt];
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[2][mt], b[0][nt], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0][mt], b[2][nt], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1][mt], b[1][nt], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1][mt], b[0][nt], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0][mt], b[1][nt], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0][mt], b[0][nt], c, 0, 0, 0);
          acc[mt][nt] = c;
        }
    };
    // unrolled (the next step's fragment reads scheduled under this step's MFMAs) where the
    // registers allow: conv2's 2 x 4 tiles; conv3's 4 x 4 and the aux heads' 2 x 6 would spill
    if constexpr (MT * NTT <= 8) {
#pragma unroll
      for (int ks = 0; ks < S::KSTEPS; ++ks) kstep(ks);
    } else {
#pragma unroll 1
      for (int ks = 0; ks < S::KSTEPS; ++ks) kstep(ks);
    }
    __syncthreads();
  }
  // the workgroup's partial: lane holds column (lane & 15) of each (tap, ci) tile and rows
  // (co) 4 (lane >> 4) .. +3 of each co tile
  float* row = slab + (int64_t)blockIdx.x * CO * S::SLAB_N;
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int nt = 0; nt < NTT; ++nt) {
      const int col = (2 * wave + nt / NTW) * (G * CX) + g * CX + 16 * (nt % NTW) + (lane & 15);
#pragma unroll
      for (int r = 0; r < 4; ++r) row[(int64_t)(16 * mt + 4 * Gq + r) * S::SLAB_N + col] = acc[mt][nt][r];
    }
  if (S::BIAS && g == 0) {  // bias partial: the threads of each channel quad, summed in a fixed order
    *reinterpret_cast<f4*>(red + 4 * tid) = dbs;
    __syncthreads();
    if (tid < CO) {
      const int c4 = tid >> 2, e = tid & 3;
      float s = 0.0f;
      for (int k = 0; k < NT / C4; ++k) s += red[4 * (c4 + C4 * k) + e];
      row[(int64_t)(4 * c4 + e) * S::SLAB_N + S::SLAB_N - 1] = s;
    }
  }
}

template <class S>
inline int launch_conv_wgrad_x6(const float* dz, const float* X, int n, float* slab, int64_t slab_cap, float* dW,
                                float* db, hipStream_t st, FrameList fl = FrameList{}, const int32_t* gdelta = nullptr) {
  const void* kfn = (const void*)conv_wgrad_x6_kernel<S>;
  VN_HIP(ensure_dyn_lds(kfn, S::LDS));
  const int items = (n + S::IMG - 1) / S::IMG * S::NB;
  constexpr int kParts = 32;
  const int64_t nel = (int64_t)S::CO * S::SLAB_N;
  int bx = std::max(1, std::min(items, resident_blocks(kfn, 512, S::LDS) / S::G));
  bx = (int)std::max<int64_t>(1, std::min<int64_t>(bx, slab_cap / nel - kParts));
  hipLaunchKernelGGL((conv_wgrad_x6_kernel<S>), dim3(bx, S::G), dim3(512), S::LDS, st, dz, X, slab, n, fl, gdelta);
  const float* src = slab;
  int nsrc = bx;
  if (bx >= 2 * kParts) {  // two-stage fixed-order reduce: one pass over hundreds of slabs is latency-bound
    float* part = slab + (int64_t)bx * nel;
    hipLaunchKernelGGL(slab_partial_kernel, dim3((unsigned)((nel + 255) / 256), kParts), dim3(256), 0, st, slab, bx, nel,
                       part);
    src = part;
    nsrc = kParts;
  }
  hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((unsigned)((nel + 255) / 256)), dim3(256), 0, st, src, nsrc, S::CO,
                     S::SLAB_N, S::KW, dW, S::BIAS ? db : nullptr, nullptr);
  return VN_OK;
}

// conv3: whole 9x9 / 3x3 dZ3 maps, images packed to >= 32 reduction pixels per item; maps
// whose planes do not fit (300x400: 17x23 under 36x48 X2) in bands of one dZ3 row (4 X2 rows),
// two images per item (46 reduction pixels, 114 KB of planes)
template <int IH, int IW, int OH, int OW>
using Conv3WgWhole = WgSpec<IH, IW, OH, OW, 64, 2, OH, (OH * OW >= 32 ? 1 : 32 / (OH * OW))>;
template <int IH, int IW, int OH, int OW>
using Conv3Wg = std::conditional_t<Conv3WgWhole<IH, IW, OH, OW>::fits, Conv3WgWhole<IH, IW, OH, OW>,
                                   WgSpec<IH, IW, OH, OW, 64, 2, 1, 2>>;
// conv2: frames (image and goal) as images; bands of 4 dZ2 rows at 174x174 (X1 rows 10 x 42),
// whole maps at 84x84; at 300x400 bands of one dZ2 row (48 reduction pixels, the 4 X1 rows of
// 99 under it: 109 KB of planes)
template <int IH, int IW, int OH, int OW>
using Conv2WgWide = WgSpec<IH, IW, OH, OW, 32, 1, (OH % 4 == 0 && OH > 9 ? 4 : OH), 1>;
template <int IH, int IW, int OH, int OW>
using Conv2Wg = std::conditional_t<Conv2WgWide<IH, IW, OH, OW>::fits, Conv2WgWide<IH, IW, OH, OW>,
                                   WgSpec<IH, IW, OH, OW, 32, 1, 1, 1>>;

template <int COUT, int CIN, int H, int W, int OH, int OW, int PY, int PX>
inline void dgrad_class_groups(const float* dz, const float* WT, float* out, const float* X, int nimg, int G,
                               hipStream_t st, int mask_goal = 1) {
  // only the covered pixels: at 84x84 the 5x5 / 5x4 classes of conv3's 9x9 input shrink to
  // 4x4 (64 of 81 rows per image; the uncovered 17 are zeroed by dgrad_all_classes_groups)
  constexpr int CH = k4s2_covered<H, OH>(), CW = k4s2_covered<W, OW>();
  constexpr int HYC = (CH - PY + 1) / 2, WXC = (CW - PX + 1) / 2;
  const int M = nimg * HYC * WXC;
  DgradA<COUT, 4, 2, OH, OW, HYC, WXC> fa{dz, M};
  static_assert(CIN == 32, "conv3: two groups of 32 channels (W^T rows of 64)");
  DgradB<COUT, 4, 2, 2 * CIN> fb{WT, G * CIN, 0, PY, PX};
  EpiMaskParityG<H, W, 2, PY, PX, HYC, WXC, CIN> ep{out, X, G, mask_goal};
  launch_gemm_x6<128, 64, 32, 2, 2>(fa, fb, ep, M, G * CIN, 4 * COUT, st);
}

template <int COUT, int CIN, int H, int W, int OH, int OW>
inline int dgrad_all_classes_groups(const float* dz, const float* WT, float* out, const float* X, int nimg, int G,
                                     hipStream_t st, int mask_goal = 1) {
  constexpr int CH = k4s2_covered<H, OH>(), CW = k4s2_covered<W, OW>();
  // the covered class pixels (CH/2 x CW/2 per class when even) over the dZ3 map
  using S = ParityDg<OH, OW, CH / 2, CW / 2, COUT, 2 * CIN, 2>;
  // VN_DGRAD_GENERIC set: the four class products instead (A/B and parity checks; read per
  // call, once per backward)
  const bool generic = getenv("VN_DGRAD_GENERIC") != nullptr;
  constexpr int BY = parity_band_rows<S>();
  if (CH % 2 == 0 && CW % 2 == 0 && S::fits && COUT == 64 && CIN == 32 && G == 2 && !generic) {
    if constexpr (CH % 2 == 0 && CW % 2 == 0 && S::fits) {
      const int rc = launch_parity_dgrad_x6<S>(dz, WT, EpiDgMaskG2<H, W>{X, out, mask_goal}, nimg, st);
      if (rc != VN_OK) return rc;
    }
  } else if (CH % 2 == 0 && CW % 2 == 0 && !S::fits && BY > 0 && COUT == 64 && CIN == 32 && G == 2 && !generic) {
    if constexpr (CH % 2 == 0 && CW % 2 == 0 && !S::fits && BY > 0) {  // 300x400: bands of class rows
      const void* kfn = (const void*)parity_dgrad_band_x6_kernel<S, BY, EpiDgMaskG2<H, W>>;
      constexpr size_t lds = parity_band_lds<S, BY>();
      VN_HIP(ensure_dyn_lds(kfn, lds));
      const int items = nimg * ((S::YC + BY - 1) / BY);
      const int blocks = std::min(items, resident_blocks(kfn, S::NT, lds));
      if (blocks > 0)
        hipLaunchKernelGGL((parity_dgrad_band_x6_kernel<S, BY, EpiDgMaskG2<H, W>>), dim3(blocks), dim3(S::NT), lds, st,
                           dz, WT, EpiDgMaskG2<H, W>{X, out, mask_goal}, nimg);
    }
  } else {
    dgrad_class_groups<COUT, CIN, H, W, OH, OW, 0, 0>(dz, WT, out, X, nimg, G, st, mask_goal);
    dgrad_class_groups<COUT, CIN, H, W, OH, OW, 0, 1>(dz, WT, out, X, nimg, G, st, mask_goal);
    dgrad_class_groups<COUT, CIN, H, W, OH, OW, 1, 0>(dz, WT, out, X, nimg, G, st, mask_goal);
    dgrad_class_groups<COUT, CIN, H, W, OH, OW, 1, 1>(dz, WT, out, X, nimg, G, st, mask_goal);
  }
  if constexpr (CH < H || CW < W) {
    const int64_t total = (int64_t)nimg * G * (H * W - CH * CW) * (CIN / 4);
    hipLaunchKernelGGL((zero_uncovered_kernel<H, W, CH, CW>), dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st,
                       out, nimg * G, CIN);
  }
  return VN_OK;
}

template <int COUT, int CINF, int H, int W, int OH, int OW>
inline void dgrad_all_classes(const float* dz, const float* WT, float* out, const float* X, int nimg, int g, int G,
                              int cin, hipStream_t st) {
  dgrad_class<COUT, CINF, H, W, OH, OW, 0, 0>(dz, WT, out, X, nimg, g, G, cin, st);
  dgrad_class<COUT, CINF, H, W, OH, OW, 0, 1>(dz, WT, out, X, nimg, g, G, cin, st);
  dgrad_class<COUT, CINF, H, W, OH, OW, 1, 0>(dz, WT, out, X, nimg, g, G, cin, st);
  dgrad_class<COUT, CINF, H, W, OH, OW, 1, 1>(dz, WT, out, X, nimg, g, G, cin, st);
}

// Frames small enough for the LDS-staged conv1 kernels (84x84, 174x174; not 300x400).
template <int H0, int W0>
constexpr bool kConv1LdsFrame = (size_t)H0 * W0 * 3 <= 96 * 1024;

template <int H0, int W0>
struct Geo {
  static constexpr int OH1 = (H0 - 7) / 4 + 1, OW1 = (W0 - 7) / 4 + 1;
  static constexpr int OH2 = (OH1 - 4) / 2 + 1, OW2 = (OW1 - 4) / 2 + 1;
  static constexpr int OH3 = (OH2 - 4) / 2 + 1, OW3 = (OW2 - 4) / 2 + 1;
  static constexpr int FCIN = 32 * OH3 * OW3;
};

// Activation store of `cap` samples: [conv1 ReLU bitmask | X1 | X2 | X3 | X4 | X5], each
// region sample-contiguous (X5 last: the recurrent core reads it as [cap][512]).
struct Acts {
  float* X[5];
  uint32_t* M1;  // [frames][OH1*OW1] channel bits of X1 > 0 (written by conv1, read by conv2's dgrad)
  int64_t off;   // samples of the buffer before X[i] (goal runs may point back to them)
};

inline Acts acts_at(const PolicyLayout& L, float* base, int64_t cap, int64_t off) {
  Acts a;
  a.off = off;
  a.M1 = reinterpret_cast<uint32_t*>(base) + off * L.msz;
  float* p = base + cap * L.msz;
  for (int i = 0; i < 5; ++i) {
    a.X[i] = p + off * L.sz[i];
    p += cap * L.sz[i];
  }
  return a;
}

// Goal-frame deduplication (vn_goal_runs) needs every frame-level kernel of the geometry to
// take a frame list: the u8 conv1 x3 kernels, the x6 / ring conv2 forward, the conv2 x6
// input gradient and weight gradient, conv3's parity-class input gradient (84x84, 174x174).
template <int H0, int W0>
constexpr bool kGoalRunsGeo = (H0 == 84 && W0 == 84) || (H0 == 174 && W0 == 174) || (H0 == 300 && W0 == 400);

inline bool goal_runs_ok(const PolicyLayout& L, int n) {
  if (L.arch != 0 || n <= kSkinnyRows) return false;
  if (!((L.H == 84 && L.W == 84) || (L.H == 174 && L.W == 174) || (L.H == 300 && L.W == 400))) return false;
  // the A/B overrides select kernels without frame lists (read per call)
  for (const char* v : {"VN_WGRAD_GENERIC", "VN_DGRAD_GENERIC", "VN_CONV2F_GENERIC", "VN_CONV2F_RING1"})
    if (getenv(v)) return false;
  return true;
}

template <int H0, int W0>
int forward_impl(const PolicyLayout& L, const float* P, const FrameSrc& src, int n, const Acts& a, float* out,
                 hipStream_t st, const vn_goal_runs* gr = nullptr) {
  using G = Geo<H0, W0>;
  const int A1 = L.A + 1;
  // goal runs: the goal frames of run starts only (checked by the caller: goal_runs_ok, u8 frames)
  const FrameList fl = gr ? FrameList{gr->goal_list, gr->goal_count, n} : FrameList{};
  // conv1 (frames -> X1), 2n frames. u8 frames take the split-bf16 kernel (bands of
  // output rows staged in LDS), else the f32 LDS-frame kernel; dense float frames take the
  // generic im2col path.
  constexpr bool kX3 = conv1_x3_fits<H0, W0>(), kConv1Lds = kConv1LdsFrame<H0, W0>;
  const bool f32in = src.f32[0] || src.f32[1];
  const int frames = 2 * n;
  bool conv1_done = false, conv2_done = false;
  if constexpr (H0 == 174 && W0 == 174) {
    // a few envs (the logged run's 4): conv1 + conv2 in one launch, one workgroup per (frame,
    // band) item (conv12_small_kernel); VN_CONV12_SMALL_OFF keeps the two launches (A/B, parity)
    if (!f32in && n <= kSkinnyRows && !gr && !getenv("VN_CONV12_SMALL_OFF")) {
      const void* kfn = (const void*)conv12_small_kernel;
      VN_HIP(ensure_dyn_lds(kfn, Conv12Small174::LDS));
      hipLaunchKernelGGL(conv12_small_kernel, dim3(frames * Conv2Ring42::NB), dim3(512), Conv12Small174::LDS, st, src,
                         frames, P + L.l[0].w, P + L.l[0].b, P + L.l[1].w, P + L.l[1].b, a.X[0], a.M1, a.X[1]);
      conv1_done = conv2_done = true;
    }
  }
  if constexpr (kX3) {
    if (!f32in && !conv1_done) {  // bf16 MFMA on split weights (exact products)
      using B = Conv1X3Band<H0, W0>;
      // weights resident in registers; VN_CONV1F_LDSW keeps the LDS-fragment kernel (A/B, parity)
      const bool ldsw = getenv("VN_CONV1F_LDSW") != nullptr;
      const void* kfn = ldsw ? (const void*)conv1_fwd_x3_kernel<H0, W0, G::OH1, G::OW1>
                             : (const void*)conv1_fwd_x3r_kernel<H0, W0, G::OH1, G::OW1>;
      const int blocks = std::min(frames * B::NB, resident_blocks(kfn, 256, 0));
      if (ldsw)
        hipLaunchKernelGGL((conv1_fwd_x3_kernel<H0, W0, G::OH1, G::OW1>), dim3(blocks), dim3(256), 0, st, src, frames,
                           fl, P + L.l[0].w, P + L.l[0].b, a.X[0], a.M1);
      else
        hipLaunchKernelGGL((conv1_fwd_x3r_kernel<H0, W0, G::OH1, G::OW1>), dim3(blocks), dim3(256), 0, st, src,
                           frames, fl, P + L.l[0].w, P + L.l[0].b, a.X[0], a.M1);
      conv1_done = true;
    }
  } else if constexpr (kConv1Lds) {
    if (!f32in && !conv1_done) {
      constexpr int NF = (2 * H0 * W0 * 3 <= 64 * 1024) ? 2 : 1;
      const int blocks = std::min((frames + NF - 1) / NF,
                                  resident_blocks((const void*)conv1_fwd_kernel<H0, W0, G::OH1, G::OW1, NF>, 320, 0));
      hipLaunchKernelGGL((conv1_fwd_kernel<H0, W0, G::OH1, G::OW1, NF>), dim3(blocks), dim3(320), 0, st, src, frames,
                         P + L.l[0].w, P + L.l[0].b, a.X[0], a.M1);
      conv1_done = true;
    }
  }
  if (!conv1_done) {
    FramesIm2col<H0, W0, G::OH1, G::OW1> fa{src, 2 * n * G::OH1 * G::OW1};
    DenseRows fb{P + L.l[0].w, 148, 32};
    EpiBiasAct ep{a.X[0], 32, P + L.l[0].b, 1};
    launch_gemm_x6<128, 32, 32, 4, 1>(fa, fb, ep, fa.M, 32, 148, st);
  }
  // conv2 (X1 -> X2): X1 bands split once into LDS planes (conv2_fwd_x6_kernel)
  if (conv2_done) {
  } else if constexpr (conv2_fwd_x6_fits<G::OH1, G::OW1, G::OH2, G::OW2>()) {
    using Bd = Conv2FwdBand<G::OH1, G::OW1, G::OH2, G::OW2>;
    const void* kfn = (const void*)conv2_fwd_x6_kernel<G::OH1, G::OW1, G::OH2, G::OW2>;
    VN_HIP(ensure_dyn_lds(kfn, Bd::LDS));  // > 64 KiB dynamic LDS: opt-in
    const int blocks = std::min(frames * Bd::NB, resident_blocks(kfn, 512, Bd::LDS));
    hipLaunchKernelGGL((conv2_fwd_x6_kernel<G::OH1, G::OW1, G::OH2, G::OW2>), dim3(blocks), dim3(512), Bd::LDS, st,
                       a.X[0], P + L.l[1].w, P + L.l[1].b, a.X[1], frames, fl);
  } else {
    using Bd = Conv2FwdBand<G::OH1, G::OW1, G::OH2, G::OW2>;
    bool done = false;
    if constexpr (conv2_fwd_ring_fits<G::OH1, G::OW1, G::OH2, G::OW2>()) {
      // training batches at 174x174: frames streamed band by band through the X1 row ring
      // (every X1 value loaded and split once); VN_CONV2F_GENERIC keeps the im2col product
      const bool generic = getenv("VN_CONV2F_GENERIC") != nullptr;  // read per call (A/B and parity checks)
      if (n > kSkinnyRows && !generic) {
        if (getenv("VN_CONV2F_RING1")) {  // the one-workgroup-per-CU form (A/B)
          const void* kfn = (const void*)conv2_fwd_ring_kernel;
          VN_HIP(ensure_dyn_lds(kfn, Conv2Ring42::LDS));
          const int blocks = std::min(frames, resident_blocks(kfn, 512, Conv2Ring42::LDS));
          hipLaunchKernelGGL(conv2_fwd_ring_kernel, dim3(blocks), dim3(512), Conv2Ring42::LDS, st, a.X[0],
                             P + L.l[1].w, P + L.l[1].b, a.X[1], frames, fl);
        } else {
          // band k + 2 prefetched through band k + 1's MFMAs; VN_CONV2F_RING2_NOPF keeps the form
          // that loads each band just before its split (A/B; bitwise equal)
          const bool pf = getenv("VN_CONV2F_RING2_NOPF") == nullptr;
          const void* kfn = pf ? (const void*)conv2_fwd_ring2_kernel<true> : (const void*)conv2_fwd_ring2_kernel<false>;
          VN_HIP(ensure_dyn_lds(kfn, Conv2Ring42x2::LDS));
          const int blocks = std::min(frames, resident_blocks(kfn, 256, Conv2Ring42x2::LDS));
          if (pf)
            hipLaunchKernelGGL(conv2_fwd_ring2_kernel<true>, dim3(blocks), dim3(256), Conv2Ring42x2::LDS, st,
                               a.X[0], P + L.l[1].w, P + L.l[1].b, a.X[1], frames, fl);
          else
            hipLaunchKernelGGL(conv2_fwd_ring2_kernel<false>, dim3(blocks), dim3(256), Conv2Ring42x2::LDS, st,
                               a.X[0], P + L.l[1].w, P + L.l[1].b, a.X[1], frames, fl);
        }
        done = true;
      }
    }
    if constexpr (Bd::LDS <= 160 * 1024) {
      // a few envs (174x174, 300x400): the banded kernel is one launch where the split-K
      // product needs two. Training batches: at 174x174 the ring above; at 300x400 the banded
      // kernel beats the generic product by 1.7-1.8 ms per update (profiles/r04/ab_conv2f.txt);
      // VN_CONV2F_GENERIC keeps the product (A/B and parity checks)
      constexpr bool ring = conv2_fwd_ring_fits<G::OH1, G::OW1, G::OH2, G::OW2>();
      if (!done && (n <= kSkinnyRows || (!ring && !getenv("VN_CONV2F_GENERIC")))) {
        const void* kfn = (const void*)conv2_fwd_x6_kernel<G::OH1, G::OW1, G::OH2, G::OW2>;
        VN_HIP(ensure_dyn_lds(kfn, Bd::LDS));
        const int blocks = std::min(frames * Bd::NB, resident_blocks(kfn, 512, Bd::LDS));
        hipLaunchKernelGGL((conv2_fwd_x6_kernel<G::OH1, G::OW1, G::OH2, G::OW2>), dim3(blocks), dim3(512), Bd::LDS, st,
                           a.X[0], P + L.l[1].w, P + L.l[1].b, a.X[1], frames, gr ? fl : FrameList{});
        done = true;
      }
    }
    if (!done && gr) {  // goal runs: the listed frames only (tiles past the device count return)
      FrameListIm2col<G::OH1, G::OW1, G::OH2, G::OW2> fa{a.X[0], 2 * n * G::OH2 * G::OW2, fl};
      DenseRows fb{P + L.l[1].w, 512, 32};
      EpiBiasActFrames<G::OH2, G::OW2> ep{a.X[1], P + L.l[1].b, fl};
      launch_gemm_x6<128, 32, 32, 4, 1>(fa, fb, ep, fa.M, 32, 512, st);
    } else if (!done) {
      NhwcIm2col<32, 4, 4, 2, G::OH1, G::OW1, G::OH2, G::OW2, 1> fa{a.X[0], 2 * n * G::OH2 * G::OW2};
      DenseRows fb{P + L.l[1].w, 512, 32};
      EpiBiasAct ep{a.X[1], 32, P + L.l[1].b, 1};
      launch_gemm_x6_sk<128, 32, 32, 4, 1>(fa, fb, ep, fa.M, 32, 512, st, L);
    }
  }
  // conv3 + conv4 of a few envs: one launch (vn_skinny.h)
  const bool small34 = n <= kSkinnyRows && !getenv("VN_CONV34_GENERIC");  // read per call (A/B and parity checks)
  if (small34) {
    const int M = n * G::OH3 * G::OW3;
    hipLaunchKernelGGL((conv34_small_kernel<G::OH2, G::OW2, G::OH3, G::OW3>), dim3((M + kC34Rows - 1) / kC34Rows),
                       dim3(1024), 0, st, a.X[1], M, P + L.l[2].w, P + L.l[2].b, P + L.l[3].w, P + L.l[3].b, a.X[2],
                       a.X[3]);
  }
  // conv3 over concat(image, goal) (X2 -> X3); with goal runs the goal half of a sample is
  // read from its run start
  if (!small34) {
    EpiBiasAct ep{a.X[2], 64, P + L.l[2].b, 1};
    DenseRows fb{P + L.l[2].w, 1024, 64};
    auto conv3 = [&](auto fa) {
      if constexpr (G::OH3 * G::OW3 >= 64)  // 174x174, 300x400: 128-row tiles (A split over more MFMAs)
        launch_gemm_x6_sk<128, 64, 32, 2, 2>(fa, fb, ep, fa.M, 64, 1024, st, L);
      else  // 84x84: 3x3 maps, 64-row tiles keep >= 2 tiles per CU
        launch_gemm_x6_sk<64, 64, 32, 2, 2>(fa, fb, ep, fa.M, 64, 1024, st, L);
    };
    // the gather with per-slot offsets (NhwcIm2colGoalF; goal half from the run start, or
    // from the sample itself without goal runs)
    // (16-B offsets: int32 up to 32 GB of X2 before and after X)
    const bool fast = (a.off + n) * 2 * G::OH2 * G::OW2 * 32 / 4 < ((int64_t)1 << 31) && !getenv("VN_CONV3F_GATHER");
    using Fast = NhwcIm2colGoalF<32, 4, 4, 2, G::OH2, G::OW2, G::OH3, G::OW3>;
    if (gr) {
      if constexpr (kGoalRunsGeo<H0, W0>) {
        if (fast)
          conv3(Fast{a.X[1], n * G::OH3 * G::OW3, gr->goal_delta});
        else
          conv3(NhwcIm2colGoal<32, 4, 4, 2, G::OH2, G::OW2, G::OH3, G::OW3>{a.X[1], n * G::OH3 * G::OW3, gr->goal_delta});
      }
    } else if (fast) {
      conv3(Fast{a.X[1], n * G::OH3 * G::OW3, nullptr});
    } else {
      conv3(NhwcIm2col<32, 4, 4, 2, G::OH2, G::OW2, G::OH3, G::OW3, 2>{a.X[1], n * G::OH3 * G::OW3});
    }
  }
  // conv4 1x1 (X3 -> X4)
  if (!small34) {
    DenseRows fa{a.X[2], 64, n * G::OH3 * G::OW3};
    DenseRows fb{P + L.l[3].w, 64, 32};
    EpiBiasAct ep{a.X[3], 32, P + L.l[3].b, 1};
    launch_gemm_x6<128, 32, 32, 4, 1>(fa, fb, ep, fa.M, 32, 64, st);
  }
  // conv_merge Linear (X4 flattened NHWC -> X5)
  {
    EpiBiasAct ep{a.X[4], 512, P + L.l[4].b, 1};
    if (n <= kSkinnyRows) {  // a few envs: whole-K VALU columns, no split-K pass (vn_skinny.h)
      launch_skinny(a.X[3], G::FCIN, P + L.l[4].w, G::FCIN, ep, n, 512, G::FCIN, st);
    } else {
      DenseRows fa{a.X[3], G::FCIN, n};
      DenseRows fb{P + L.l[4].w, G::FCIN, 512};
      launch_gemm_x6_sk<64, 64, 32, 2, 2, 64>(fa, fb, ep, n, 512, G::FCIN, st, L);
    }
  }
  // heads (X5 -> out[n][8]: logits, value); out == NULL runs the trunk only (recurrent policy)
  if (out) {
    EpiBiasAct ep{out, OUT_LD, P + L.l[5].b, 0};
    if (n <= kSkinnyRows) {
      launch_skinny(a.X[4], 512, P + L.l[5].w, 512, ep, n, A1, 512, st);
    } else {
      DenseRows fa{a.X[4], 512, n};
      DenseRows fb{P + L.l[5].w, 512, A1};
      launch_gemm_sk<64, 16, 32, 4, 1>(fa, fb, ep, n, A1, 512, st, L);
    }
  }
  VN_HIP(hipGetLastError());
  return VN_OK;
}

struct BwdWork {
  float* wt;
  float* dz5;
  float* dz4;
  float* dz3;
  float* dz2;
  float* slab;
  int64_t slab_cap;
};

inline int64_t slab_floats(const PolicyLayout& L) {
  return 24ll << 20;  // split-K slab capacity (launch_wgrad halves the split count to fit)
}

inline int64_t workspace_floats(const PolicyLayout& L, int64_t n) {
  return L.wt_total + n * 512 + n * L.FCIN + n * L.sz[2] + n * L.sz[1] + slab_floats(L) + 64;
}

inline BwdWork carve(const PolicyLayout& L, float* ws, int64_t n) {
  BwdWork w;
  float* p = ws;
  w.wt = p;
  p += L.wt_total;
  w.dz5 = p;
  p += n * 512;
  w.dz4 = p;
  p += n * L.FCIN;
  w.dz3 = p;
  p += n * L.sz[2];
  w.dz2 = p;
  p += n * L.sz[1];
  w.slab = p;
  w.slab_cap = slab_floats(L);
  return w;
}

template <int H0, int W0>
int backward_impl(const PolicyLayout& L, const float* P, const FrameSrc& src, int n, const Acts& a,
                  const float* dout, const float* dz5_in, const float* dx4_extra, float* Gr, const BwdWork& w,
                  hipStream_t st, const vn_goal_runs* gr = nullptr) {
  using G = Geo<H0, W0>;
  const int A1 = L.A + 1;
  // goal runs: the image frames and the goal frames of run starts (ascending)
  const FrameList fl = gr ? FrameList{gr->goal_list, gr->goal_count, n} : FrameList{};
  auto T = [&](int i) { return w.wt + L.wt_off[i]; };
  // dz5_in != NULL: the trunk backward of the recurrent policy (heads and LSTM already done)
  const float* dz5 = dz5_in ? dz5_in : w.dz5;
  {  // transposed weights for the dgrad products, one launch
    TransposeSet ts;
    for (int i = 1; i < 6; ++i) ts.add(P + L.l[i].w, L.l[i].cout, L.l[i].kp, T(i));
    launch_transpose_set(ts, st);
  }
  const int n9 = n * G::OH3 * G::OW3;
  // ---- head: dX5 = dout x Whead, masked by X5 ; dWhead = dout^T x X5
  if (!dz5_in) {
    DenseRows fa{dout, OUT_LD, n};
    DenseRows fb{T(5), A1, 512};  // WT [512][A1]
    EpiMask ep{w.dz5, a.X[4], 512};
    launch_gemm<64, 64, 32, 2, 2>(fa, fb, ep, n, 512, A1, st);
    Im2colT<DenseRows> fbw{DenseRows{a.X[4], 512, n}, 512};
    launch_wgrad<32, 64, 2, 2>(dout, OUT_LD, A1, fbw, 512, n, w.slab, w.slab_cap, Gr + L.l[5].w, Gr + L.l[5].b, st);
  }
  // ---- conv_merge Linear: dX4 = dz5 x Wfc masked by X4 ; dWfc = dz5^T x X4
  {
    DenseRows fa{dz5, 512, n};
    DenseRows fb{T(4), 512, G::FCIN};  // WT [FCIN][512]
    // 128x128 tiles for the wide maps (174x174: N = 2592, C5): half the split work per MFMA;
    // 0.2-0.4 ms per update (profiles/r05/ab_cm/); 84x84's N = 288 keeps 64x64
    // Few rows (the logged run's 4 x 20 = 80): 64x64 tiles, split-K below 128 tiles (the
    // 128x128 form ran 21 workgroups down K = 512 alone: 54 us of a 2 ms update)
    const bool big = G::FCIN >= 1024 && n >= 256;
    auto dgrad = [&](auto ep) {
      if (big)
        launch_gemm_x6<128, 128, 32, 2, 2>(fa, fb, ep, n, G::FCIN, 512, st);
      else
        launch_gemm_x6_sk<64, 64, 32, 2, 2>(fa, fb, ep, n, G::FCIN, 512, st, L);
    };
    if (dx4_extra)  // + the aux heads' gradient w.r.t. X4, under the same ReLU mask
      dgrad(EpiMaskAdd{w.dz4, a.X[3], G::FCIN, dx4_extra});
    else
      dgrad(EpiMask{w.dz4, a.X[3], G::FCIN});
    Im2colT<DenseRows> fbw{DenseRows{a.X[3], G::FCIN, n}, G::FCIN};
    launch_wgrad6<128, 128, 2, 2>(dz5, 512, 512, fbw, G::FCIN, n, w.slab, w.slab_cap, Gr + L.l[4].w, Gr + L.l[4].b,
                                  st);
  }
  // ---- conv4 (1x1): dX3 = dz4 x W4 masked by X3 ; dW4 = dz4^T x X3
  {
    DenseRows fa{w.dz4, 32, n9};
    DenseRows fb{T(3), 32, 64};  // WT [64][32]
    EpiMask ep{w.dz3, a.X[2], 64};
    launch_gemm_x6<64, 64, 32, 2, 2>(fa, fb, ep, n9, 64, 32, st);
    Im2colT<DenseRows> fbw{DenseRows{a.X[2], 64, n9}, 64};
    launch_wgrad<32, 64, 2, 2>(w.dz4, 32, 32, fbw, 64, n9, w.slab, w.slab_cap, Gr + L.l[3].w, Gr + L.l[3].b, st);
  }
  // ---- conv3 (k4 s2, 2 input groups): wgrad, then dgrad into dz2 masked by X2
  {
    using Im = NhwcIm2col<32, 4, 4, 2, G::OH2, G::OW2, G::OH3, G::OW3, 2>;
    Im2colT<Im> fbw{Im{a.X[1], n9}, 1024};
    using Wg = Conv3Wg<G::OH2, G::OW2, G::OH3, G::OW3>;
    if (Wg::fits && !getenv("VN_WGRAD_GENERIC")) {  // read per call (A/B and parity checks)
      if constexpr (Wg::fits) {
        const int rc = launch_conv_wgrad_x6<Wg>(w.dz3, a.X[1], n, w.slab, w.slab_cap, Gr + L.l[2].w, Gr + L.l[2].b, st,
                                                FrameList{}, gr ? gr->goal_delta : nullptr);
        if (rc != VN_OK) return rc;
      }
    } else if (gr) {  // goal runs: the goal half of a sample's X2 at its run start
      if constexpr (kGoalRunsGeo<H0, W0>) {
        using ImG = NhwcIm2colGoal<32, 4, 4, 2, G::OH2, G::OW2, G::OH3, G::OW3>;
        Im2colT<ImG> fbg{ImG{a.X[1], n9, gr->goal_delta}, 1024};
        launch_wgrad6<64, 128, 2, 2>(w.dz3, 64, 64, fbg, 1024, n9, w.slab, w.slab_cap, Gr + L.l[2].w, Gr + L.l[2].b,
                                     st);
      }
    } else {
      launch_wgrad6<64, 128, 2, 2>(w.dz3, 64, 64, fbw, 1024, n9, w.slab, w.slab_cap, Gr + L.l[2].w, Gr + L.l[2].b, st);
    }
    const int rc =
        dgrad_all_classes_groups<64, 32, G::OH2, G::OW2, G::OH3, G::OW3>(w.dz3, T(2), w.dz2, a.X[1], n, 2, st, gr ? 0 : 1);
    if (rc != VN_OK) return rc;
    if (gr) {  // each run's goal-map gradient: summed over the run at its start, masked there
      constexpr int64_t frame_f4 = (int64_t)G::OH2 * G::OW2 * 8;
      const int blocks = (int)std::min<int64_t>((n * frame_f4 + 255) / 256, 4096);
      hipLaunchKernelGGL(goal_dz2_reduce_kernel, dim3(blocks), dim3(256), 0, st, w.dz2, a.X[1], frame_f4, gr->goal_list,
                         gr->goal_count, gr->run_length, gr->num_envs);
    }
  }
  // ---- conv2 (k4 s2): wgrad (needs X1), then dgrad into dz1 written over X1
  {
    const int frames = 2 * n;
    using Bd2 = Conv2WgBand<G::OH1, G::OW1, G::OH2, G::OW2>;
    const int blocks = std::min(frames * Bd2::NB, kConv2WgradBlocks);
    constexpr size_t lds = conv2_wgrad_lds<G::OH1, G::OW1, G::OH2, G::OW2>();
    using Wg2 = Conv2Wg<G::OH1, G::OW1, G::OH2, G::OW2>;
    // x6 form; VN_WGRAD_GENERIC / VN_CONV2WG_F32 (this product only) keep the others (A/B and
    // parity checks; read per call)
    if (Wg2::fits && !getenv("VN_WGRAD_GENERIC") && !getenv("VN_CONV2WG_F32")) {
      if constexpr (Wg2::fits) {
        const int rc = launch_conv_wgrad_x6<Wg2>(w.dz2, a.X[0], frames, w.slab, w.slab_cap, Gr + L.l[1].w, Gr + L.l[1].b,
                                                 st, fl);
        if (rc != VN_OK) return rc;
      }
    } else if constexpr (lds <= 80 * 1024) {  // f32 MFMA, two workgroups per CU (bands of output rows)
      VN_HIP(ensure_dyn_lds((const void*)conv2_wgrad_kernel<G::OH1, G::OW1, G::OH2, G::OW2>, lds));  // > 64 KiB dynamic LDS: opt-in
      float* bias_slab = w.slab + (int64_t)blocks * 32 * 512;
      hipLaunchKernelGGL((conv2_wgrad_kernel<G::OH1, G::OW1, G::OH2, G::OW2>), dim3(blocks), dim3(256), lds, st,
                         a.X[0], w.dz2, frames, w.slab, bias_slab, fl);
      // two-stage fixed-order reduce of the per-workgroup slabs (one pass over 512 slabs per
      // element ran 118 us, latency-bound)
      constexpr int kParts = 32;
      float* part = bias_slab + (int64_t)blocks * 32;
      float* bpart = part + (int64_t)kParts * 32 * 512;
      hipLaunchKernelGGL(slab_partial_kernel, dim3((32 * 512 + 255) / 256, kParts), dim3(256), 0, st, w.slab, blocks,
                         (int64_t)32 * 512, part);
      hipLaunchKernelGGL(slab_partial_kernel, dim3(1, kParts), dim3(32), 0, st, bias_slab, blocks, (int64_t)32, bpart);
      hipLaunchKernelGGL(sum_slabs_kernel, dim3((32 * 512 + 255) / 256), dim3(256), 0, st, part, kParts,
                         (int64_t)32 * 512, Gr + L.l[1].w);
      hipLaunchKernelGGL(sum_slabs_kernel, dim3(1), dim3(32), 0, st, bpart, kParts, (int64_t)32, Gr + L.l[1].b);
    } else {  // a conv1 map row too wide for a band in half the LDS: generic split-K path
      using Im = NhwcIm2col<32, 4, 4, 2, G::OH1, G::OW1, G::OH2, G::OW2, 1>;
      const int P2 = 2 * n * G::OH2 * G::OW2;
      Im2colT<Im> fbw{Im{a.X[0], P2}, 512};
      launch_wgrad<32, 64, 2, 2>(w.dz2, 32, 32, fbw, 512, P2, w.slab, w.slab_cap, Gr + L.l[1].w, Gr + L.l[1].b, st);
    }
    if constexpr (G::OH1 % 2 == 0 && G::OW1 % 2 == 0) {
      // the u8 conv1 kernel left X1's ReLU as a bitmask: read 4 B per pixel instead of X1
      const bool bits = (conv1_x3_fits<H0, W0>() || kConv1LdsFrame<H0, W0>) && !(src.f32[0] || src.f32[1]);
      bool done = false;
      if constexpr (conv2_dgrad_x6_fits<G::OH1, G::OW1, G::OH2, G::OW2>()) {
        if (bits) {
          constexpr int NW = conv2_dgrad_x6_waves<G::OH1, G::OW1, G::OH2, G::OW2>();
          // the rotated item loop (ROT) by default; VN_CONV2DG_NOROT keeps the original (A/B,
          // bitwise equal). Lanes past the class map store to a 16-B sink in the slab (free
          // here: conv2's weight gradient has been reduced, conv1's starts after this kernel)
          const bool rot = getenv("VN_CONV2DG_NOROT") == nullptr;
          const void* kfn = rot ? (const void*)conv2_dgrad_x6_kernel<G::OH1, G::OW1, G::OH2, G::OW2, NW, true>
                                : (const void*)conv2_dgrad_x6_kernel<G::OH1, G::OW1, G::OH2, G::OW2, NW, false>;
          constexpr size_t lds = conv2_dgrad_x6_lds<G::OH1, G::OW1, G::OH2, G::OW2>();
          VN_HIP(ensure_dyn_lds(kfn, lds));  // > 64 KiB dynamic LDS: opt-in
          const int blocks = std::min(frames, resident_blocks(kfn, NW * 64, lds));
          if (rot)
            hipLaunchKernelGGL((conv2_dgrad_x6_kernel<G::OH1, G::OW1, G::OH2, G::OW2, NW, true>), dim3(blocks),
                               dim3(NW * 64), lds, st, w.dz2, T(1), a.M1, a.X[0], frames, fl, w.slab);
          else
            hipLaunchKernelGGL((conv2_dgrad_x6_kernel<G::OH1, G::OW1, G::OH2, G::OW2, NW, false>), dim3(blocks),
                               dim3(NW * 64), lds, st, w.dz2, T(1), a.M1, a.X[0], frames, fl, w.slab);
          done = true;
        }
      }
      if (done) {
      } else if (bits) {
        const int blocks = std::min(
            frames, resident_blocks((const void*)conv2_dgrad_kernel<G::OH1, G::OW1, G::OH2, G::OW2, true>, 256, 0));
        hipLaunchKernelGGL((conv2_dgrad_kernel<G::OH1, G::OW1, G::OH2, G::OW2, true>), dim3(blocks), dim3(256), 0, st,
                           w.dz2, T(1), a.X[0], a.M1, a.X[0], frames);
      } else {
        const int blocks = std::min(
            frames, resident_blocks((const void*)conv2_dgrad_kernel<G::OH1, G::OW1, G::OH2, G::OW2, false>, 256, 0));
        hipLaunchKernelGGL((conv2_dgrad_kernel<G::OH1, G::OW1, G::OH2, G::OW2, false>), dim3(blocks), dim3(256), 0, st,
                           w.dz2, T(1), a.X[0], a.M1, a.X[0], frames);
      }
    } else {
      // odd conv1 maps (300x400: 74x99): the banded x6 kernel over the u8 conv1 bitmask; the
      // four class products for float frames or under VN_DGRAD_GENERIC (A/B, parity tests)
      const bool bits = conv1_x3_fits<H0, W0>() && !(src.f32[0] || src.f32[1]) && !getenv("VN_DGRAD_GENERIC");
      if (bits) {
        constexpr int BY = conv2_dgrad_band_rows<G::OW1, G::OW2>();
        using Bd = Conv2DgBand<G::OH1, G::OW1, G::OH2, G::OW2, BY>;
        const void* kfn = (const void*)conv2_dgrad_band_x6_kernel<G::OH1, G::OW1, G::OH2, G::OW2, BY>;
        VN_HIP(ensure_dyn_lds(kfn, Bd::LDS));
        const int blocks = std::min(frames * Bd::NB, resident_blocks(kfn, 256, Bd::LDS));
        hipLaunchKernelGGL((conv2_dgrad_band_x6_kernel<G::OH1, G::OW1, G::OH2, G::OW2, BY>), dim3(blocks), dim3(256),
                           Bd::LDS, st, w.dz2, T(1), a.M1, a.X[0], frames, fl);
      } else {
        dgrad_all_classes<32, 32, G::OH1, G::OW1, G::OH2, G::OW2>(w.dz2, T(1), a.X[0], a.X[0], 2 * n, 0, 1, 32, st);
      }
    }
  }
  // ---- conv1: wgrad from dz1 (in X1's storage) and the frames
  constexpr bool kConv1Lds = kConv1LdsFrame<H0, W0>;
  const bool f32in = src.f32[0] || src.f32[1];
  bool wg_done = false;
  if constexpr (conv1_wgrad_x3_fits<H0, W0>()) {
    if (!f32in) {
      const int frames = 2 * n;
      using Bd = Conv1WgBand<H0, W0>;
      // LEAN (scalar lane masks, no per-step B masking; bitwise equal) where it keeps its SGPRs:
      // 174x174 and 300x400 (the 84x84 instance spills 34 SGPRs); VN_CONV1WG_NOLEAN for A/B
      constexpr bool kLean = !(H0 == 84 && W0 == 84);
      const bool lean = kLean && getenv("VN_CONV1WG_NOLEAN") == nullptr;
      const void* kfn = lean ? (const void*)conv1_wgrad_x3_kernel<H0, W0, G::OH1, G::OW1, kLean>
                             : (const void*)conv1_wgrad_x3_kernel<H0, W0, G::OH1, G::OW1, false>;
      const size_t lds = Bd::LDS + (lean ? 16 : 0);  // + the bias lane's 8 bf16 ones
      const int blocks = std::min(frames * Bd::NB, resident_blocks(kfn, 256, lds));
      if (lean)
        hipLaunchKernelGGL((conv1_wgrad_x3_kernel<H0, W0, G::OH1, G::OW1, kLean>), dim3(blocks), dim3(256), lds, st,
                           src, frames, fl, a.X[0], w.slab);
      else
        hipLaunchKernelGGL((conv1_wgrad_x3_kernel<H0, W0, G::OH1, G::OW1, false>), dim3(blocks), dim3(256), lds, st,
                           src, frames, fl, a.X[0], w.slab);
      constexpr int kParts = 32;
      float* part = w.slab + (int64_t)blocks * 32 * 160;
      hipLaunchKernelGGL(slab_partial_kernel, dim3((32 * 160 + 255) / 256, kParts), dim3(256), 0, st, w.slab, blocks,
                         (int64_t)32 * 160, part);
      hipLaunchKernelGGL(conv1_wgrad_x3_finish_kernel, dim3((32 * 160 + 255) / 256), dim3(256), 0, st, part, kParts,
                         (int)Bd::Q::ID, Gr + L.l[0].w, Gr + L.l[0].b);
      wg_done = true;
    }
  } else if constexpr (kConv1Lds) {
    if (!f32in) {
      const int frames = 2 * n;
      constexpr int CP = (G::OH1 * G::OW1 <= 400) ? (G::OH1 * G::OW1 + 7) / 8 * 8 : 448;
      constexpr size_t lds = conv1_wgrad_lds<H0, W0, CP>();
      VN_HIP(ensure_dyn_lds((const void*)conv1_wgrad_kernel<H0, W0, G::OH1, G::OW1, CP>, lds));  // > 64 KiB dynamic LDS: opt-in
      const int blocks = std::min({frames, kConv1WgradBlocks,
                                   resident_blocks((const void*)conv1_wgrad_kernel<H0, W0, G::OH1, G::OW1, CP>, 256, lds)});
      hipLaunchKernelGGL((conv1_wgrad_kernel<H0, W0, G::OH1, G::OW1, CP>), dim3(blocks), dim3(256), lds, st, src, frames,
                         a.X[0], w.slab);
      hipLaunchKernelGGL(conv1_wgrad_reduce_kernel, dim3((32 * 160 + 255) / 256), dim3(256), 0, st, w.slab, blocks * 4,
                         Gr + L.l[0].w, Gr + L.l[0].b);
      wg_done = true;
    }
  }
  if (!wg_done) {
    using Im = FramesIm2col<H0, W0, G::OH1, G::OW1>;
    const int P1 = 2 * n * G::OH1 * G::OW1;
    Im2colT<Im> fbw{Im{src, P1}, 148};
    launch_wgrad<32, 64, 2, 2>(a.X[0], 32, 32, fbw, 148, P1, w.slab, w.slab_cap, Gr + L.l[0].w, Gr + L.l[0].b, st);
  }
  VN_HIP(hipGetLastError());
  return VN_OK;
}

// ---- BigHouseModel trunk (models/bignet.py:26-41,70-75): image only ---------------------
template <int H0, int W0>
int forward_bignet(const PolicyLayout& L, const float* P, const FrameSrc& src, int n, const Acts& a, float* out,
                   hipStream_t st) {
  constexpr int OH1 = (H0 - 8) / 4 + 1, OW1 = (W0 - 8) / 4 + 1;
  constexpr int OH2 = (OH1 - 4) / 2 + 1, OW2 = (OW1 - 4) / 2 + 1;
  constexpr int OH3 = OH2 - 2, OW3 = OW2 - 2, FCIN = 32 * OH3 * OW3;
  {  // conv1 3 -> 32, k8 s4 (X1 [n][OH1][OW1][32])
    FramesIm2colK8<H0, W0, OH1, OW1> fa{src, n * OH1 * OW1};
    DenseRows fb{P + L.l[0].w, 192, 32};
    EpiBiasAct ep{a.X[0], 32, P + L.l[0].b, 1};
    launch_gemm_x6<128, 32, 32, 4, 1>(fa, fb, ep, fa.M, 32, 192, st);
  }
  {  // conv2 32 -> 64, k4 s2
    NhwcIm2col<32, 4, 4, 2, OH1, OW1, OH2, OW2, 1> fa{a.X[0], n * OH2 * OW2};
    DenseRows fb{P + L.l[1].w, 512, 64};
    EpiBiasAct ep{a.X[1], 64, P + L.l[1].b, 1};
    launch_gemm_x6<64, 64, 32, 2, 2>(fa, fb, ep, fa.M, 64, 512, st);
  }
  {  // conv3 64 -> 32, k3 s1
    NhwcIm2col<64, 3, 3, 1, OH2, OW2, OH3, OW3, 1> fa{a.X[1], n * OH3 * OW3};
    DenseRows fb{P + L.l[2].w, 576, 32};
    EpiBiasAct ep{a.X[2], 32, P + L.l[2].b, 1};
    launch_gemm_x6<128, 32, 32, 4, 1>(fa, fb, ep, fa.M, 32, 576, st);
  }
  {  // conv_merge Linear(32*7*7 -> 512) + ReLU (X5)
    DenseRows fa{a.X[2], FCIN, n};
    DenseRows fb{P + L.l[4].w, FCIN, 512};
    EpiBiasAct ep{a.X[4], 512, P + L.l[4].b, 1};
    launch_gemm_x6_sk<64, 64, 32, 2, 2, 64>(fa, fb, ep, n, 512, FCIN, st, L);
  }
  if (out) {
    DenseRows fa{a.X[4], 512, n};
    DenseRows fb{P + L.l[5].w, 512, L.A + 1};
    EpiBiasAct ep{out, OUT_LD, P + L.l[5].b, 0};
    launch_gemm_sk<64, 16, 32, 4, 1>(fa, fb, ep, n, L.A + 1, 512, st, L);
  }
  VN_HIP(hipGetLastError());
  return VN_OK;
}

template <int H0, int W0>
int backward_bignet(const PolicyLayout& L, const float* P, const FrameSrc& src, int n, const Acts& a,
                    const float* dout, const float* dz5_in, const float* dx3_extra, float* Gr, const BwdWork& w,
                    hipStream_t st) {
  constexpr int OH1 = (H0 - 8) / 4 + 1, OW1 = (W0 - 8) / 4 + 1;
  constexpr int OH2 = (OH1 - 4) / 2 + 1, OW2 = (OW1 - 4) / 2 + 1;
  constexpr int OH3 = OH2 - 2, OW3 = OW2 - 2, FCIN = 32 * OH3 * OW3;
  const int A1 = L.A + 1;
  auto T = [&](int i) { return w.wt + L.wt_off[i]; };
  {
    TransposeSet ts;
    for (int i = 1; i < 6; ++i) ts.add(P + L.l[i].w, L.l[i].cout, L.l[i].kp, T(i));
    launch_transpose_set(ts, st);
  }
  const float* dz5 = dz5_in ? dz5_in : w.dz5;
  if (!dz5_in) {  // heads
    DenseRows fa{dout, OUT_LD, n};
    DenseRows fb{T(5), A1, 512};
    EpiMask ep{w.dz5, a.X[4], 512};
    launch_gemm<64, 64, 32, 2, 2>(fa, fb, ep, n, 512, A1, st);
    Im2colT<DenseRows> fbw{DenseRows{a.X[4], 512, n}, 512};
    launch_wgrad<32, 64, 2, 2>(dout, OUT_LD, A1, fbw, 512, n, w.slab, w.slab_cap, Gr + L.l[5].w, Gr + L.l[5].b, st);
  }
  float* dz3 = w.dz4;  // [n][FCIN]
  float* dz2 = w.dz2;  // [n][OH2*OW2*64]
  {  // conv_merge: dX3 = dz5 x Wfc (+ reward prediction's dX3) masked by X3 ; dWfc
    DenseRows fa{dz5, 512, n};
    DenseRows fb{T(4), 512, FCIN};
    if (dx3_extra) {
      EpiMaskAdd ep{dz3, a.X[2], FCIN, dx3_extra};
      launch_gemm_x6<64, 64, 32, 2, 2>(fa, fb, ep, n, FCIN, 512, st);
    } else {
      EpiMask ep{dz3, a.X[2], FCIN};
      launch_gemm_x6<64, 64, 32, 2, 2>(fa, fb, ep, n, FCIN, 512, st);
    }
    Im2colT<DenseRows> fbw{DenseRows{a.X[2], FCIN, n}, FCIN};
    launch_wgrad6<128, 128, 2, 2>(dz5, 512, 512, fbw, FCIN, n, w.slab, w.slab_cap, Gr + L.l[4].w, Gr + L.l[4].b, st);
  }
  {  // conv3 (k3 s1): wgrad, then the single-class dgrad into dz2 masked by X2
    using Im = NhwcIm2col<64, 3, 3, 1, OH2, OW2, OH3, OW3, 1>;
    const int P3 = n * OH3 * OW3;
    launch_wgrad<32, 64, 2, 2>(dz3, 32, 32, Im2colT<Im>{Im{a.X[1], P3}, 576}, 576, P3, w.slab, w.slab_cap,
                               Gr + L.l[2].w, Gr + L.l[2].b, st);
    const int M = n * OH2 * OW2;
    DgradA<32, 3, 1, OH3, OW3, OH2, OW2> fa{dz3, M};
    DgradB<32, 3, 1, 64> fb{T(2), 64, 0, 0, 0};
    EpiMaskParity<OH2, OW2, 1, 0, 0, OH2, OW2> ep{dz2, a.X[1], 0, 1, 64};
    launch_gemm_x6<64, 64, 32, 2, 2>(fa, fb, ep, M, 64, 9 * 32, st);
  }
  {  // conv2 (k4 s2): wgrad, then parity-class dgrad over X1 in place
    using Im = NhwcIm2col<32, 4, 4, 2, OH1, OW1, OH2, OW2, 1>;
    const int P2 = n * OH2 * OW2;
    launch_wgrad6<64, 128, 2, 2>(dz2, 64, 64, Im2colT<Im>{Im{a.X[0], P2}, 512}, 512, P2, w.slab, w.slab_cap,
                               Gr + L.l[1].w, Gr + L.l[1].b, st);
    dgrad_all_classes<64, 32, OH1, OW1, OH2, OW2>(dz2, T(1), a.X[0], a.X[0], n, 0, 1, 32, st);
  }
  {  // conv1 wgrad from dX1 (in X1's storage) and the frames
    using Im = FramesIm2colK8<H0, W0, OH1, OW1>;
    const int P1 = n * OH1 * OW1;
    launch_wgrad<32, 64, 2, 2>(a.X[0], 32, 32, Im2colT<Im>{Im{src, P1}, 192}, 192, P1, w.slab, w.slab_cap,
                               Gr + L.l[0].w, Gr + L.l[0].b, st);
  }
  VN_HIP(hipGetLastError());
  return VN_OK;
}

// ---- recurrent core (vn_lstm.h) --------------------------------------------------
inline int lstm_forward_step(const PolicyLayout& L, const float* P, int E, const float* x5, const float* lra,
                             const float* mask, const float* h_prev, const float* c_prev, float* xc, float* gates,
                             float* acts, float* c_out, float* h_out, hipStream_t st) {
  if (E <= kSkinnyRows) {  // xcat build + gates + cell in one launch (vn_skinny.h)
    XcatFill xf{x5, lra, mask, h_prev, L.A + 1, L.xoff};
    const dim3 grid(256), block(256);  // 2 hidden units (8 gate columns) per workgroup
    if (E <= 4)
      hipLaunchKernelGGL(lstm_step_skinny_kernel<4>, grid, block, 0, st, xf, E, L.xcat, P + L.lw, P + L.lbih,
                         P + L.lbhh, c_prev, xc, acts, c_out, h_out);
    else if (E <= 8)
      hipLaunchKernelGGL(lstm_step_skinny_kernel<8>, grid, block, 0, st, xf, E, L.xcat, P + L.lw, P + L.lbih,
                         P + L.lbhh, c_prev, xc, acts, c_out, h_out);
    else
      hipLaunchKernelGGL(lstm_step_skinny_kernel<kSkinnyRows>, grid, block, 0, st, xf, E, L.xcat, P + L.lw,
                         P + L.lbih, P + L.lbhh, c_prev, xc, acts, c_out, h_out);
    VN_HIP(hipGetLastError());
    return VN_OK;
  }
  const int64_t nx = (int64_t)E * L.xcat;
  hipLaunchKernelGGL(lstm_prep_kernel, dim3((unsigned)((nx + 255) / 256)), dim3(256), 0, st, E, L.A, L.xcat, L.xoff,
                     x5, lra, mask, h_prev, xc);
  {
    DenseRows fa{xc, L.xcat, E};
    DenseRows fb{P + L.lw, L.xcat, 2048};
    EpiBias2 ep{gates, 2048, P + L.lbih, P + L.lbhh};
    launch_gemm_x6_sk<128, 128, 32, 2, 2>(fa, fb, ep, E, 2048, L.xcat, st, L);
  }
  const int64_t nc = (int64_t)E * 512;
  hipLaunchKernelGGL(lstm_cell_kernel, dim3((unsigned)((nc + 255) / 256)), dim3(256), 0, st, E, gates, c_prev, mask,
                     acts, c_out, h_out);
  VN_HIP(hipGetLastError());
  return VN_OK;
}

inline int heads_forward(const PolicyLayout& L, const float* P, const float* feat, int n, float* out, hipStream_t st) {
  EpiBiasAct ep{out, OUT_LD, P + L.l[5].b, 0};
  if (n <= kSkinnyRows) {
    launch_skinny(feat, 512, P + L.l[5].w, 512, ep, n, L.A + 1, 512, st);
  } else {
    DenseRows fa{feat, 512, n};
    DenseRows fb{P + L.l[5].w, 512, L.A + 1};
    launch_gemm_sk<64, 16, 32, 4, 1>(fa, fb, ep, n, L.A + 1, 512, st, L);
  }
  VN_HIP(hipGetLastError());
  return VN_OK;
}

struct LstmWork {
  float* wcat_t;   // [xcat][2048]
  float* head_t;   // [512][A+1]
  float* dh_heads; // [T*E][512]
  float* dgates;   // [T*E][2048]
  float* dh[2];    // [E][512]
  float* dc[2];    // [E][512]
  float* slab;
};

inline int64_t lstm_workspace_floats(const PolicyLayout& L, int64_t T, int64_t E) {
  const int64_t n = T * E;
  return 2048ll * L.xcat + 512ll * 8 + n * 512 + n * 2048 + 4 * E * 512 + slab_floats(L) + 64;
}

inline LstmWork lstm_carve(const PolicyLayout& L, float* ws, int64_t T, int64_t E) {
  LstmWork w;
  float* p = ws;
  w.wcat_t = p;
  p += 2048ll * L.xcat;
  w.head_t = p;
  p += 512ll * 8;
  w.dh_heads = p;
  p += T * E * 512;
  w.dgates = p;
  p += T * E * 2048;
  for (int i = 0; i < 2; ++i) {
    w.dh[i] = p;
    p += E * 512;
    w.dc[i] = p;
    p += E * 512;
  }
  w.slab = p;
  return w;
}

// BPTT over one rollout of T steps x E envs (rows t*E + e), from dL/d(out) [T*E][8].
// Writes the head and LSTM gradients into Gr and dL/dX5 (masked by conv_merge's ReLU)
// into dz5 for the trunk backward.
inline int lstm_backward(const PolicyLayout& L, const float* P, int T, int E, const float* dout, const float* h_all,
                         const float* xcat_all, const float* acts_all, const float* c_all, const float* c_init,
                         const float* mask_all, const float* x5_all, float* dz5, float* Gr, const LstmWork& w,
                         hipStream_t st, const float* dh_extra = nullptr, int extra_envs = 0) {
  const int A1 = L.A + 1;
  const int N = T * E;
  const int64_t e512 = (int64_t)E * 512;
  {
    TransposeSet ts;
    ts.add(P + L.lw, 2048, L.xcat, w.wcat_t);
    ts.add(P + L.l[5].w, A1, 512, w.head_t);
    launch_transpose_set(ts, st);
  }
  {  // heads: dh_heads = dout x Whead ; dWhead = dout^T x h
    DenseRows fa{dout, OUT_LD, N};
    DenseRows fb{w.head_t, A1, 512};
    EpiStore ep{w.dh_heads, 512};
    launch_gemm<64, 64, 32, 2, 2>(fa, fb, ep, N, 512, A1, st);
    Im2colT<DenseRows> fbw{DenseRows{h_all, 512, N}, 512};
    launch_wgrad<32, 64, 2, 2>(dout, OUT_LD, A1, fbw, 512, N, w.slab, slab_floats(L), Gr + L.l[5].w, Gr + L.l[5].b,
                               st);
  }
  if (dh_extra) {  // the output gradient of other heads on the first extra_envs envs (pixel control)
    const int64_t total = (int64_t)T * extra_envs * 128;
    hipLaunchKernelGGL(add_env_rows_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, dh_extra, T, E,
                       extra_envs, 512, w.dh_heads);
  }
  const unsigned cb = (unsigned)((e512 + 255) / 256);
  if (E <= kSkinnyRows) {
    // a few envs: the cell backward of the last step, then per step t one launch with the
    // sequential product dh_{t-1} = m_t (dgates_t W_hh) and step t-1's cell backward
    // (dh_{-1} is not needed: no launch for t = 0)
    {
      const int t = T - 1;
      hipLaunchKernelGGL(lstm_cell_bwd_kernel, dim3(cb), dim3(256), 0, st, E, w.dh_heads + (int64_t)t * e512, nullptr,
                         nullptr, acts_all + (int64_t)t * E * 2048, c_all + (int64_t)t * e512,
                         t > 0 ? c_all + (int64_t)(t - 1) * e512 : c_init, mask_all ? mask_all + (int64_t)t * E : nullptr,
                         w.dgates + (int64_t)t * E * 2048, w.dc[0]);
    }
    for (int t = T - 1, cur = 0; t >= 1; --t, cur ^= 1) {
      LstmBwdStep p;
      p.dgates_t = w.dgates + (int64_t)t * E * 2048;
      p.whh_t = w.wcat_t + (int64_t)L.xoff * 2048;
      p.mask_t = mask_all ? mask_all + (int64_t)t * E : nullptr;
      p.dh_heads = w.dh_heads + (int64_t)(t - 1) * e512;
      p.dc_next = w.dc[cur];
      p.acts = acts_all + (int64_t)(t - 1) * E * 2048;
      p.c = c_all + (int64_t)(t - 1) * e512;
      p.c_prev = t - 1 > 0 ? c_all + (int64_t)(t - 2) * e512 : c_init;
      p.mask_prev = mask_all ? mask_all + (int64_t)(t - 1) * E : nullptr;
      p.dgates_prev = w.dgates + (int64_t)(t - 1) * E * 2048;
      p.dc_prev_out = w.dc[cur ^ 1];
      const dim3 grid(512 / kSkCols);
      if (E <= 4)
        hipLaunchKernelGGL(lstm_bwd_skinny_kernel<4>, grid, dim3(256), 0, st, p, E);
      else if (E <= 8)
        hipLaunchKernelGGL(lstm_bwd_skinny_kernel<8>, grid, dim3(256), 0, st, p, E);
      else
        hipLaunchKernelGGL(lstm_bwd_skinny_kernel<kSkinnyRows>, grid, dim3(256), 0, st, p, E);
    }
  }
  for (int t = T - 1, cur = 0; t >= 0 && E > kSkinnyRows; --t, cur ^= 1) {
    const bool last = (t == T - 1);
    const float* mask = mask_all ? mask_all + (int64_t)t * E : nullptr;
    const float* cprev = t > 0 ? c_all + (int64_t)(t - 1) * e512 : c_init;
    float* dg = w.dgates + (int64_t)t * E * 2048;
    hipLaunchKernelGGL(lstm_cell_bwd_kernel, dim3(cb), dim3(256), 0, st, E, w.dh_heads + (int64_t)t * e512,
                       last ? nullptr : w.dh[cur ^ 1], last ? nullptr : w.dc[cur ^ 1], acts_all + (int64_t)t * E * 2048,
                       c_all + (int64_t)t * e512, cprev, mask, dg, w.dc[cur]);
    // only the recurrent part is sequential: dh_{t-1} = m_t (dgates_t x W_hh)
    DenseRows fa{dg, 2048, E};
    DenseRows fb{w.wcat_t + (int64_t)L.xoff * 2048, 2048, 512};
    EpiLstmDh ep{w.dh[cur], mask};
    launch_gemm_x6_sk<64, 64, 32, 2, 2, 64>(fa, fb, ep, E, 512, 2048, st, L);
  }
  {  // the trunk's input gradient of all T steps in one product: dz5 = relu'(x5) (dgates x W_ih[:, :512])
    DenseRows fa{w.dgates, 2048, N};
    DenseRows fb{w.wcat_t, 2048, 512};
    EpiMask ep{dz5, x5_all, 512};
    // split-K below 128 tiles: the logged run's 80 rows make 4 tiles, each walking K = 2048
    // alone (0.14 ms, 6 % of its update); bench batches have thousands of tiles and run as before
    launch_gemm_x6_sk<128, 128, 32, 2, 2>(fa, fb, ep, N, 512, 2048, st, L);
  }
  {  // dW_cat = dgates^T x xcat over all T*E rows (x6 core, both operands staged k-major from
     // their [rows][*] stores); b_ih and b_hh share the bias gradient
    if (getenv("VN_LSTM_WG_TRANSPOSED")) {
      // A/B switch: the former form on tile_transpose'd copies, in stream-ordered scratch of
      // its own (the workspace no longer carries the 2 x T*E x (2048 + xcat) floats)
      const int64_t nt = ((int64_t)N + 3) / 4 * 4;
      float* tt = nullptr;
      VN_HIP(hipMallocAsync((void**)&tt, (size_t)nt * (2048 + L.xcat) * sizeof(float), st));
      float* dgt = tt;
      float* xct = tt + nt * 2048;
      tile_transpose(w.dgates, N, 2048, 2048, dgt, nt, st);
      tile_transpose(xcat_all, N, L.xcat, L.xcat, xct, nt, st);
      launch_wgrad_x6<128, 128, 2, 2>(dgt, 2048, xct, L.xcat, N, nt, w.slab, slab_floats(L), Gr + L.lw, Gr + L.lbih,
                                     st, Gr + L.lbhh);
      VN_HIP(hipFreeAsync(tt, st));
    } else {
      launch_wgrad_x6t<128, 128, 2, 2>(w.dgates, 2048, 2048, xcat_all, L.xcat, L.xcat, N, w.slab, slab_floats(L),
                                      Gr + L.lw, Gr + L.lbih, st, Gr + L.lbhh);
    }
  }
  VN_HIP(hipGetLastError());
  return VN_OK;
}

// ---- aux deconv heads (vn_aux.h) ---------------------------------------------------
// One parity class (PY, PX) of a k4 s2 transposed conv in [n][IH][IW][CIN] -> out
// [n][OH][OW][COUT] (OH = 2 IH + 2): the trunk's dgrad loaders with a bias/ReLU epilogue.
template <int CIN, int COUT, int IH, int IW, int OH, int OW, int PY, int PX>
inline void deconv_class(const float* in, const float* WT, float* out, const float* bias, int relu, int nimg,
                         hipStream_t st) {
  constexpr int HYC = OH / 2, WXC = OW / 2;
  const int M = nimg * HYC * WXC;
  DgradA<CIN, 4, 2, IH, IW, HYC, WXC> fa{in, M};
  DgradB<CIN, 4, 2, COUT> fb{WT, COUT, 0, PY, PX};
  EpiDeconv<OH, OW, PY, PX, HYC, WXC> ep{out, COUT, bias, relu};
  if constexpr (COUT >= 32)
    launch_gemm_x6<64, 64, 32, 2, 2>(fa, fb, ep, M, COUT, 4 * CIN, st);
  else
    launch_gemm<64, 16, 32, 4, 1>(fa, fb, ep, M, COUT, 4 * CIN, st);
}

template <int CIN, int COUT, int IH, int IW, int OH, int OW>
inline int deconv_all(const float* in, const float* WT, float* out, const float* bias, int relu, int nimg,
                       hipStream_t st) {
  static_assert(OH == 2 * IH + 2 && OW == 2 * IW + 2, "k4 s2 transposed conv geometry");
  // the first layers (aux heads 32 -> 48: one wave per class; pixel control 32 -> 64: two)
  // on the persistent parity-class kernel
  constexpr bool kPc = COUT == 64;
  using S = ParityDg<IH, IW, OH / 2, OW / 2, 32, kPc ? 64 : 48, kPc ? 2 : 1>;
  if constexpr (CIN == 32 && (COUT == 48 || COUT == 64) && S::fits) {
    if (!getenv("VN_DGRAD_GENERIC")) {  // read per call (A/B and parity checks)
      const int rc = launch_parity_dgrad_x6<S>(in, WT, EpiDgBias<OH, OW, COUT>{out, bias, relu}, nimg, st);
      if (rc != VN_OK) return rc;
      return VN_OK;
    }
  }
  deconv_class<CIN, COUT, IH, IW, OH, OW, 0, 0>(in, WT, out, bias, relu, nimg, st);
  deconv_class<CIN, COUT, IH, IW, OH, OW, 0, 1>(in, WT, out, bias, relu, nimg, st);
  deconv_class<CIN, COUT, IH, IW, OH, OW, 1, 0>(in, WT, out, bias, relu, nimg, st);
  deconv_class<CIN, COUT, IH, IW, OH, OW, 1, 1>(in, WT, out, bias, relu, nimg, st);
  return VN_OK;
}

struct AuxWork {
  float* w1t;    // [16*48][32]
  float* w2t;    // [16*8][48]
  float* slab;
  float* colsum; // [kColsumBlocks][48]
  float* db;     // [48] scratch (the ones-column output of the weight-gradient products)
};
constexpr int kColsumBlocks = 512;

inline int64_t aux_workspace_floats(const PolicyLayout& L) {
  return 768ll * 32 + 128ll * 48 + slab_floats(L) + (int64_t)kColsumBlocks * 48 + 64 + 64;
}

inline AuxWork aux_carve(const PolicyLayout& L, float* ws) {
  AuxWork w;
  float* p = ws;
  w.w1t = p;
  p += 768ll * 32;
  w.w2t = p;
  p += 128ll * 48;
  w.slab = p;
  p += slab_floats(L);
  w.colsum = p;
  p += (int64_t)kColsumBlocks * 48;
  w.db = p;
  return w;
}

inline void colsum(const float* src, int64_t rows, int cols, float* partial, float* out, hipStream_t st) {
  const int lanes = 256 / cols;
  const int blocks = (int)std::max<int64_t>(1, std::min<int64_t>(kColsumBlocks, (rows + lanes - 1) / lanes));
  hipLaunchKernelGGL(colsum_partial_kernel, dim3(blocks), dim3(256), 0, st, src, rows, cols, partial);
  hipLaunchKernelGGL(colsum_final_kernel, dim3(cols), dim3(64), 0, st, partial, blocks, cols, out);
}

template <int AH, int AW, int PH, int PW, bool LOSS>
inline void launch_aux2(const float* A1, int n, const float* W2, const float* b2, float* pred,
                        const vn_aux_targets* tg, float weight, float* dpred, float* stats, hipStream_t st) {
  constexpr size_t lds = aux2_lds<AH, AW>();
  const void* kfn = (const void*)aux_deconv2_kernel<AH, AW, PH, PW, LOSS>;
  (void)ensure_dyn_lds(kfn, lds);  // > 64 KiB dynamic LDS: opt-in (a failure surfaces at the launch check)
  constexpr int SPI = aux2_spi<AH, AW>();
  const int blocks = std::min((n + SPI - 1) / SPI, resident_blocks(kfn, kAux2Threads, lds));
  hipLaunchKernelGGL((aux_deconv2_kernel<AH, AW, PH, PW, LOSS>), dim3(blocks), dim3(kAux2Threads), lds, st, A1, n, W2,
                     b2, pred, tg ? reinterpret_cast<const f4*>(tg->table) : nullptr, tg ? tg->image_rows : nullptr,
                     tg ? tg->goal_rows : nullptr, weight, dpred, stats);
}

// The banded second layer (maps too large for aux_deconv2_kernel's whole-map staging).
template <int AH, int AW, int PH, int PW, bool LOSS>
inline void launch_aux2_band(const float* A1, int n, const float* W2, const float* b2, float* pred,
                             const vn_aux_targets* tg, float weight, float* dpred, float* stats, hipStream_t st) {
  constexpr int BYC = aux2_byc<AW, PW>();
  constexpr size_t lds = aux2b_lds(AW, BYC);
  const void* kfn = (const void*)aux_deconv2_band_kernel<AH, AW, PH, PW, LOSS, BYC>;
  (void)ensure_dyn_lds(kfn, lds);
  const int items = n * ((PH / 2 + BYC - 1) / BYC);
  const int blocks = std::min(items, resident_blocks(kfn, kAux2Threads, lds));
  hipLaunchKernelGGL((aux_deconv2_band_kernel<AH, AW, PH, PW, LOSS, BYC>), dim3(blocks), dim3(kAux2Threads), lds, st,
                     A1, n, W2, b2, pred, tg ? reinterpret_cast<const f4*>(tg->table) : nullptr,
                     tg ? tg->image_rows : nullptr, tg ? tg->goal_rows : nullptr, weight, dpred, stats);
}

template <int H0, int W0>
int aux_forward_impl(const PolicyLayout& L, const float* P, const float* X4, int n, float* A1, float* Pout,
                     const AuxWork& w, hipStream_t st) {
  using G = Geo<H0, W0>;
  constexpr int IH = G::OH3, IW = G::OW3, AH = 2 * IH + 2, AW = 2 * IW + 2, PH = 2 * AH + 2, PW = 2 * AW + 2;
  {
    TransposeSet ts;
    ts.add(P + L.aw1, 32, 768, w.w1t);
    ts.add(P + L.aw2, 48, 128, w.w2t);
    launch_transpose_set(ts, st);
  }
  if (const int rc = deconv_all<32, kAuxC1, IH, IW, AH, AW>(X4, w.w1t, A1, P + L.ab1, 1, n, st); rc != VN_OK) return rc;
  if constexpr (aux2_fits<AH, AW>()) {
    launch_aux2<AH, AW, PH, PW, false>(A1, n, P + L.aw2, P + L.ab2, Pout, nullptr, 0.0f, nullptr, nullptr, st);
  } else if constexpr (aux2_byc<AW, PW>() > 0) {
    launch_aux2_band<AH, AW, PH, PW, false>(A1, n, P + L.aw2, P + L.ab2, Pout, nullptr, 0.0f, nullptr, nullptr, st);
  } else {
    if (const int rc = deconv_all<kAuxC1, kAuxC2, AH, AW, PH, PW>(A1, w.w2t, Pout, P + L.ab2, 0, n, st); rc != VN_OK) return rc;
  }
  VN_HIP(hipGetLastError());
  return VN_OK;
}

// Forward of both head layers with the loss fused into the second: dpred and stats as
// vn_aux_loss_grad, the prediction itself is not written (maps whose A1 does not fit the
// direct kernel's LDS run forward + loss separately into `pred`).
template <int H0, int W0>
int aux_forward_loss_impl(const PolicyLayout& L, const float* P, const float* X4, int n, float* A1, float* pred,
                          const vn_aux_targets* tg, float weight, float* dpred, float* stats, const AuxWork& w,
                          hipStream_t st) {
  using G = Geo<H0, W0>;
  constexpr int IH = G::OH3, IW = G::OW3, AH = 2 * IH + 2, AW = 2 * IW + 2, PH = 2 * AH + 2, PW = 2 * AW + 2;
  if constexpr (aux2_fits<AH, AW>() || aux2_byc<AW, PW>() > 0) {
    hipLaunchKernelGGL(transpose_kernel, dim3((32 * 768 + 255) / 256), dim3(256), 0, st, P + L.aw1, 32, 768, w.w1t);
    if (const int rc = deconv_all<32, kAuxC1, IH, IW, AH, AW>(X4, w.w1t, A1, P + L.ab1, 1, n, st); rc != VN_OK) return rc;
    if constexpr (aux2_fits<AH, AW>())
      launch_aux2<AH, AW, PH, PW, true>(A1, n, P + L.aw2, P + L.ab2, nullptr, tg, weight, dpred, stats, st);
    else
      launch_aux2_band<AH, AW, PH, PW, true>(A1, n, P + L.aw2, P + L.ab2, nullptr, tg, weight, dpred, stats, st);
  } else {
    const int rc = aux_forward_impl<H0, W0>(L, P, X4, n, A1, pred, w, st);
    if (rc != VN_OK) return rc;
    hipLaunchKernelGGL(aux_loss_grad_kernel, dim3(kAuxLossBlocks), dim3(256), 0, st, n, PH, PW, pred,
                       reinterpret_cast<const f4*>(tg->table), tg->image_rows, tg->goal_rows, weight, dpred, stats);
  }
  VN_HIP(hipGetLastError());
  return VN_OK;
}

// Second head layer backward as products (maps whose dP does not fit aux_backward2_kernel's
// LDS): dW2 = A1^T x im2col(dP) (block-diagonal mask), db2 = column sums of dP (the head
// biases come from column sums, so the weight products carry no ones column), dA1 =
// conv(dP, W2) masked by the ReLU of A1 in place, db1 = column sums of dA1.
template <int AH, int AW, int PH, int PW>
void aux_backward_layer2_gemm(const PolicyLayout& L, const float* P, int n, float* A1, const float* dP, float* Gr,
                              const AuxWork& w, hipStream_t st) {
  const int P1 = n * AH * AW;
  using Im2 = NhwcIm2col<kAuxC2, 4, 4, 2, PH, PW, AH, AW, 1>;  // dP windows per A1 pixel
  launch_wgrad6<64, 128, 2, 2>(A1, kAuxC1, kAuxC1, Im2colT<Im2>{Im2{dP, P1}, 16 * kAuxC2}, 16 * kAuxC2, P1, w.slab,
                               slab_floats(L), Gr + L.aw2, nullptr, st);
  hipLaunchKernelGGL(aux_blockdiag_mask_kernel, dim3((kAuxC1 * 16 * kAuxC2 + 255) / 256), dim3(256), 0, st,
                     Gr + L.aw2);
  colsum(dP, (int64_t)n * PH * PW, kAuxC2, w.colsum, Gr + L.ab2, st);
  {
    DenseRows fb{P + L.aw2, 16 * kAuxC2, kAuxC1};
    EpiMask ep{A1, A1, kAuxC1};
    launch_gemm_x6<64, 64, 32, 2, 2>(Im2{dP, P1}, fb, ep, P1, kAuxC1, 16 * kAuxC2, st);
  }
  colsum(A1, (int64_t)P1, kAuxC1, w.colsum, Gr + L.ab1, st);
}

// dX4 = conv(dA1, W1) (k4 s2, 48 -> 32 channels: the aux heads' first layer's input gradient)
// as a persistent parity-class product, in place of the generic im2col product (which re-splits
// every dA1 value at each of its 4 uses and the weights in every workgroup). A work item is a
// band of BY output rows of one sample (the whole 9x9 / 3x3 map at 174x174 / 84x84; 3 rows at
// 300x400, whose 17x23 map does not fit): its dA1 rows are split once into three bf16 planes
// per parity class (py, px) = (y & 1, x & 1): class pixel (oy0 + cyl, cx) at row cyl XC + cx
// (XC = IW + 1), 48 channels a row, class rows past the map stored as zeros. Output pixel (oy, ox)
// of the consecutive-row index p = oy XC + ox (ox = IW: a dummy column) sums, per class, the
// taps (ky, kx) = (py + 2 ty, px + 2 tx), which read class rows p + ty XC + tx: 16 consecutive
// rows per 16-pixel tile and tap. Wave w owns class w >> 1 and output channels 16 (w & 1) ..
// +15; its split weights (4 taps x 48 channels x 16 columns x 3 terms) stay in registers. The
// product is transposed (MFMA rows = output channels, columns = pixels, 16x16x32, six k steps
// of 32 over the class's 4 taps x 48 channels); after each tile the four class partials meet in
// LDS (double-buffered by tile parity) and are summed in class order by all 512 threads.
template <int AH, int AW, int IH, int IW>
struct AuxDx4 {
  static constexpr int C = kAuxC1, CO = 32;
  static constexpr int XC = IW + 1, YC = IH + 1;
  static constexpr int PP = 36;  // partial row stride (floats)
  static constexpr int TG = 2;   // tiles per partial-sum round (one barrier)
  static constexpr int tp_of(int by) { return (by * XC + 15) / 16 * 16; }  // tiled output rows
  static constexpr int nr_of(int by) { return tp_of(by) + XC + 1; }        // plane rows: the last tile's reads
  static constexpr size_t lds_of(int by) { return (size_t)12 * nr_of(by) * C * 2 + (size_t)2 * TG * 4 * 16 * PP * 4; }
  static constexpr int by_max() {
    int by = IH;
    while (by > 1 && lds_of(by) > 160 * 1024) --by;
    return by;
  }
  // a band of BY output rows stages class rows oy0 .. oy0 + BY (dA1 rows 2 oy0 .. 2 oy0 + 2 BY + 1)
  static constexpr int BY = by_max(), NB = (IH + BY - 1) / BY, SR = BY + 1;
  static constexpr int TP = tp_of(BY), NR = nr_of(BY), PL = NR * C;
  static constexpr int NS = 2 * SR * AW * (C / 4);  // staged f4 per item
  static constexpr int NV = (NS + 511) / 512;       // prefetched f4 per thread
  static constexpr size_t LDS = lds_of(BY);
  static constexpr bool fits = LDS <= 160 * 1024 && AH == 2 * IH + 2 && AW == 2 * IW + 2;
};

template <int AH, int AW, int IH, int IW>
__global__ __launch_bounds__(512, 1) void aux_dx4_x6_kernel(const float* __restrict__ dA1,
                                                             const float* __restrict__ W1, float* __restrict__ dX4,
                                                             int n) {
  using S = AuxDx4<AH, AW, IH, IW>;
  constexpr int C = S::C, XC = S::XC, TP = S::TP, NR = S::NR, PL = S::PL, PP = S::PP, NV = S::NV, NS = S::NS;
  constexpr int BY = S::BY, NB = S::NB, SR = S::SR;
  constexpr int C4 = C / 4, TILES = TP / 16, TG = S::TG;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem_adx[];
  uint16_t* pl = reinterpret_cast<uint16_t*>(smem_adx);            // [term][class][NR][C]
  float* part = reinterpret_cast<float*>(smem_adx + (size_t)12 * PL * 2);  // [2][TG][class][16][PP]
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int cls = wave >> 1, ch = wave & 1, py = cls >> 1, px = cls & 1;
  const int i16 = lane & 15, q = lane >> 4;
  // split weights: step s, lane (co = 16 ch + i16, q) holds k' = 32 s + 8 q .. +7 of the class's
  // local K (tap t = k' / 48 = 2 ty + tx, channel k' % 48)
  bf16x8_t bw[6][3];
#pragma unroll
  for (int st = 0; st < 6; ++st) {
    const int kl = 32 * st + 8 * q, t = kl / C, c0 = kl - (kl / C) * C;
    const int ky = py + 2 * (t >> 1), kx = px + 2 * (t & 1);
    const float* w = W1 + (int64_t)(16 * ch + i16) * (16 * C) + (ky * 4 + kx) * C + c0;
    union { uint16_t u[8]; bf16x8_t v; } b0, b1, b2;
#pragma unroll
    for (int j = 0; j < 8; ++j) split3_bf16(w[j], b0.u[j], b1.u[j], b2.u[j]);
    bw[st][0] = b0.v;
    bw[st][1] = b1.v;
    bw[st][2] = b2.v;
  }
  // plane rows past the staged class rows (the last tiles' reads) stay zero; every item
  // rewrites rows 0 .. SR XC - 1 (zeros for class rows past the map)
  for (int i = tid; i < 12 * (NR - SR * XC) * C4 / 2; i += 512) {
    const int per = (NR - SR * XC) * C4 / 2, pln = i / per, r = i - pln * per;
    reinterpret_cast<uint4*>(pl + (size_t)pln * PL + SR * XC * C)[r] = uint4{0u, 0u, 0u, 0u};
  }
  const int items = n * NB;
  f4 pre[NV];
  auto load = [&](int it) {  // dA1 rows 2 oy0 .. of item it (rows past the map: any row, stored as 0)
    const int smp = it / NB, b = it - (it / NB) * NB;
    const f4* src = reinterpret_cast<const f4*>(dA1 + (int64_t)smp * AH * AW * C);
    const int f0 = 2 * BY * b * AW * C4, fend = AH * AW * C4;
#pragma unroll
    for (int j = 0; j < NV; ++j) pre[j] = src[min(f0 + min(tid + j * 512, NS - 1), fend - 1)];  // unconditional
  };
  if ((int)blockIdx.x < items) load(blockIdx.x);
  int par = 0;  // partial-buffer parity (rounds run so far)
  for (int it = blockIdx.x; it < items; it += gridDim.x) {
    const int smp = it / NB, b = it - (it / NB) * NB, oy0 = BY * b, nr = min(BY, IH - oy0);
    __syncthreads();  // the previous item's plane reads are done
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      const int i = tid + j * 512;
      if (i < NS) {
        const int pix = i / C4, c4 = i - (i / C4) * C4, yl = pix / AW, x = pix - (pix / AW) * AW;
        uint2 t0, t1, t2;
        split3_pack(2 * oy0 + yl < AH ? pre[j] : f4zero(), t0, t1, t2);
        uint16_t* d = pl + (size_t)((yl & 1) * 2 + (x & 1)) * PL + ((yl >> 1) * XC + (x >> 1)) * C + 4 * c4;
        *reinterpret_cast<uint2*>(d) = t0;
        *reinterpret_cast<uint2*>(d + 4 * PL) = t1;
        *reinterpret_cast<uint2*>(d + 8 * PL) = t2;
      }
    }
    __syncthreads();
    load(min(it + (int)gridDim.x, items - 1));
    const uint16_t* cp = pl + (size_t)cls * PL;
#pragma unroll 1
    for (int t0 = 0; t0 < TILES; t0 += TG) {
      // TG tiles per round: independent accumulators, one barrier for their partials
      f4 acc[TG];
#pragma unroll
      for (int u = 0; u < TG; ++u) acc[u] = f4zero();
#pragma unroll
      for (int st = 0; st < 6; ++st) {
        const int kl = 32 * st + 8 * q, t = kl / C, c0 = kl - (kl / C) * C;
#pragma unroll
        for (int u = 0; u < TG; ++u) {
          // a tile past the map (odd TILES) recomputes the last one; its partials are unused
          const int row = min(t0 + u, TILES - 1) * 16 + i16 + (t >> 1) * XC + (t & 1);
          bf16x8_t a[3];
#pragma unroll
          for (int tm = 0; tm < 3; ++tm)
            a[tm] = *reinterpret_cast<const bf16x8_t*>(cp + (size_t)tm * 4 * PL + row * C + c0);
          f4 c = acc[u];
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bw[st][0], a[2], c, 0, 0, 0);  // small terms first
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bw[st][2], a[0], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bw[st][1], a[1], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bw[st][0], a[1], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bw[st][1], a[0], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bw[st][0], a[0], c, 0, 0, 0);
          acc[u] = c;
        }
      }
      // lane (pixel i16, q) holds output channels 16 ch + 4q .. +3 of its tile pixel
      float* pb = part + (size_t)par * TG * 4 * 16 * PP;
#pragma unroll
      for (int u = 0; u < TG; ++u)
        *reinterpret_cast<f4*>(pb + ((u * 4 + cls) * 16 + i16) * PP + 16 * ch + 4 * q) = acc[u];
      __syncthreads();
#pragma unroll
      for (int u = 0; u < TG; ++u) {  // (pixel, channel): the four class partials in class order
        const float* pu = pb + (size_t)u * 4 * 16 * PP;
        const int pi = tid >> 5, co = tid & 31, pp = (t0 + u) * 16 + pi, oyl = pp / XC, ox = pp - (pp / XC) * XC;
        const float v = ((pu[pi * PP + co] + pu[(16 + pi) * PP + co]) + pu[(32 + pi) * PP + co]) + pu[(48 + pi) * PP + co];
        if (t0 + u < TILES && oyl < nr && ox < IW)
          dX4[(((int64_t)smp * IH + oy0 + oyl) * IW + ox) * S::CO + co] = v;
      }
      par ^= 1;
    }
  }
}

// Gradients of the heads' parameters and dX4 [n][IH][IW][32] (unmasked) from dP; A1 is
// overwritten by its own gradient.
template <int H0, int W0>
int aux_backward_impl(const PolicyLayout& L, const float* P, const float* X4, int n, float* A1, const float* dP,
                      float* Gr, float* dX4, const AuxWork& w, hipStream_t st) {
  using G = Geo<H0, W0>;
  constexpr int IH = G::OH3, IW = G::OW3, AH = 2 * IH + 2, AW = 2 * IW + 2, PH = 2 * AH + 2, PW = 2 * AW + 2;
  const int P0 = n * IH * IW;
  using Im1 = NhwcIm2col<kAuxC1, 4, 4, 2, AH, AW, IH, IW, 1>;  // dA1 windows per X4 pixel
  if constexpr (auxb_fits<AH, AW, PH, PW>()) {
    // second layer in one pass: dW2, db2, dA1 (masked, over A1) and db1
    const void* kfn = (const void*)aux_backward2_kernel<AH, AW, PH, PW>;
    constexpr size_t lds = auxb_lds<PH, PW>();
    VN_HIP(ensure_dyn_lds(kfn, lds));  // > 64 KiB dynamic LDS: opt-in
    const int blocks = std::min(n, std::min(resident_blocks(kfn, kAuxBThreads, lds), kColsumBlocks));
    hipLaunchKernelGGL((aux_backward2_kernel<AH, AW, PH, PW>), dim3(blocks), dim3(kAuxBThreads), lds, st, A1, dP, n,
                       P + L.aw2, w.slab);
    hipLaunchKernelGGL(aux_backward2_finish_kernel, dim3((kAuxC1 * 16 * kAuxC2 + kAuxC1 + kAuxC2 + 3) / 4),
                       dim3(256), 0, st, w.slab, blocks, Gr + L.aw2, Gr + L.ab1, Gr + L.ab2);
  } else if constexpr (auxb_bya<AH, AW, PH, PW>() > 0) {
    // the same pass in bands of A1 rows (300x400: 8 rows over 18 dP rows, 64 KB)
    constexpr int BYA = auxb_bya<AH, AW, PH, PW>();
    const void* kfn = (const void*)aux_backward2_kernel<AH, AW, PH, PW, BYA>;
    constexpr size_t lds = auxb_band_lds(PW, BYA);
    VN_HIP(ensure_dyn_lds(kfn, lds));
    const int items = n * ((AH + BYA - 1) / BYA);
    const int blocks = std::min(items, std::min(resident_blocks(kfn, kAuxBThreads, lds), kColsumBlocks));
    hipLaunchKernelGGL((aux_backward2_kernel<AH, AW, PH, PW, BYA>), dim3(blocks), dim3(kAuxBThreads), lds, st, A1, dP,
                       n, P + L.aw2, w.slab);
    hipLaunchKernelGGL(aux_backward2_finish_kernel, dim3((kAuxC1 * 16 * kAuxC2 + kAuxC1 + kAuxC2 + 3) / 4),
                       dim3(256), 0, st, w.slab, blocks, Gr + L.aw2, Gr + L.ab1, Gr + L.ab2);
  } else {
    aux_backward_layer2_gemm<AH, AW, PH, PW>(L, P, n, A1, dP, Gr, w, st);
  }
  // first layer: dW1 = X4^T x im2col(dA1); dX4 = conv(dA1, W1). The weight gradient is a
  // stride-2 k4 weight gradient with X4 as the reduced map and dA1 (48 channels) under it:
  // dW1[ci][tap][co] = sum X4[iy][ix][ci] dA1[2iy + ky][2ix + kx][co] (no bias column)
  using WaWhole = WgSpec<AH, AW, IH, IW, 32, 1, IH, (IH * IW >= 32 ? 1 : 32 / (IH * IW)), kAuxC1, false>;
  // maps whose planes do not fit (300x400): bands of one X4 row (4 A1 rows), two images per item
  using Wa = std::conditional_t<WaWhole::fits, WaWhole, WgSpec<AH, AW, IH, IW, 32, 1, 1, 2, kAuxC1, false>>;
  if (Wa::fits && !getenv("VN_WGRAD_GENERIC")) {  // read per call (A/B and parity checks)
    if constexpr (Wa::fits) {
      const int rc = launch_conv_wgrad_x6<Wa>(X4, A1, n, w.slab, slab_floats(L), Gr + L.aw1, nullptr, st);
      if (rc != VN_OK) return rc;
    }
  } else {
    launch_wgrad6<32, 128, 1, 4>(X4, 32, 32, Im2colT<Im1>{Im1{A1, P0}, 16 * kAuxC1}, 16 * kAuxC1, P0, w.slab,
                                 slab_floats(L), Gr + L.aw1, nullptr, st);
  }
  using Dx = AuxDx4<AH, AW, IH, IW>;
  if (Dx::fits && !getenv("VN_AUX_DX4_GENERIC")) {  // read per call (A/B and parity checks)
    if constexpr (Dx::fits) {
      const void* kfn = (const void*)aux_dx4_x6_kernel<AH, AW, IH, IW>;
      VN_HIP(ensure_dyn_lds(kfn, Dx::LDS));
      const int blocks = std::min(n * Dx::NB, resident_blocks(kfn, 512, Dx::LDS));
      if (blocks > 0)
        hipLaunchKernelGGL((aux_dx4_x6_kernel<AH, AW, IH, IW>), dim3(blocks), dim3(512), Dx::LDS, st, A1, P + L.aw1,
                           dX4, n);
    }
  } else {
    DenseRows fb{P + L.aw1, 16 * kAuxC1, 32};
    EpiStore ep{dX4, 32};
    launch_gemm_x6<128, 32, 32, 4, 1>(Im1{A1, P0}, fb, ep, P0, 32, 16 * kAuxC1, st);
  }
  VN_HIP(hipGetLastError());
  return VN_OK;
}


// ---- UNREAL heads (vn_unreal.h) -------------------------------------------------------
struct PcWork {
  float* w1t;     // [16*64][32]
  float* w2t;     // [16*8][64]
  float* wpct;    // [512][2592]
  float* slab;
  float* colsum;  // [kColsumBlocks][64]
};

inline int64_t pc_workspace_floats(const PolicyLayout& L) {
  return 1024ll * 32 + 128ll * 64 + 512ll * kPcBase + slab_floats(L) + (int64_t)kColsumBlocks * 64 + 64;
}

inline PcWork pc_carve(const PolicyLayout& L, float* ws) {
  PcWork w;
  float* p = ws;
  w.w1t = p;
  p += 1024ll * 32;
  w.w2t = p;
  p += 128ll * 64;
  w.wpct = p;
  p += 512ll * kPcBase;
  w.slab = p;
  p += slab_floats(L);
  w.colsum = p;
  return w;
}

// pixel_control (goal.py:131-137) on feature rows h [n][512]: pc_base (x6 product, bias,
// ReLU), the two first deconvs as one 32 -> 64 deconv, the two second deconvs as one
// block-diagonal 64 -> 8 deconv (ReLU on both), then the value/action combination.
// The pixel-control map's side: 42 (BigGoalHouseModel's two k4 s2 layers) or 20 (BigHouseModel's one).
inline int pc_side(const PolicyLayout& L) { return L.arch == 1 ? kPcA1 : kPcP; }

int pc_forward_impl(const PolicyLayout& L, const float* P, const float* h, int n, float* pcb, float* A1, float* P2,
                    float* q, const PcWork& w, hipStream_t st) {
  {
    DenseRows fa{h, 512, n};
    DenseRows fb{P + L.upw, 512, kPcBase};
    EpiBiasAct ep{pcb, kPcBase, P + L.upb, 1};
    launch_gemm_x6_sk<64, 64, 32, 2, 2>(fa, fb, ep, n, kPcBase, 512, st, L);
  }
  if (L.arch == 1) {  // bignet.py:105-111: pc_value / pc_action side by side as one 32 -> 8 deconv
    TransposeSet ts;
    ts.add(P + L.uw1, 32, 16 * kPcC2, w.w1t);
    launch_transpose_set(ts, st);
    if (const int rc = deconv_all<32, kPcC2, kPcMap, kPcMap, kPcA1, kPcA1>(pcb, w.w1t, P2, P + L.ub1, 1, n, st);
        rc != VN_OK)
      return rc;
  } else {
    {
      TransposeSet ts;
      ts.add(P + L.uw1, 32, 16 * kPcC1, w.w1t);
      ts.add(P + L.uw2, kPcC1, 16 * kPcC2, w.w2t);
      launch_transpose_set(ts, st);
    }
    if (const int rc = deconv_all<32, kPcC1, kPcMap, kPcMap, kPcA1, kPcA1>(pcb, w.w1t, A1, P + L.ub1, 1, n, st);
        rc != VN_OK)
      return rc;
    if (const int rc = deconv_all<kPcC1, kPcC2, kPcA1, kPcA1, kPcP, kPcP>(A1, w.w2t, P2, P + L.ub2, 1, n, st);
        rc != VN_OK)
      return rc;
  }
  if (q) {  // the trainer's pixel-control loss forms q from P2 itself
    const int64_t npix = (int64_t)n * pc_side(L) * pc_side(L);
    hipLaunchKernelGGL(pc_combine_kernel, dim3((unsigned)((npix + 255) / 256)), dim3(256), 0, st, P2, npix, L.A, q);
  }
  VN_HIP(hipGetLastError());
  return VN_OK;
}

// Gradients of the pixel-control parameters and dh [n][512] (stored, or added when
// accumulate) from dq [n][42][42][A]. Consumes P2 (-> dP2), A1 (-> dA1) and pcb (-> dpcb).
int pc_backward_impl(const PolicyLayout& L, const float* P, const float* h, int n, float* pcb, float* A1, float* P2,
                     const float* dq, float* Gr, float* dh, int accumulate, const PcWork& w, hipStream_t st) {
  const int64_t npix = (int64_t)n * pc_side(L) * pc_side(L);
  if (dq)  // else P2 already holds dL/dP2 (vn_unreal_pc_loss_grad)
    hipLaunchKernelGGL(pc_dq_kernel, dim3((unsigned)((npix + 255) / 256)), dim3(256), 0, st, P2, dq, npix, L.A);
  if (L.arch == 1) {
    // the one layer: dW1[ci][tap][co] = sum pcb[iy][ix][ci] dP2[2iy + ky][2ix + kx][co] (the
    // action and padding columns see dP2 = 0), db1, dpcb = conv(dP2, W1) under pc_base's ReLU
    const int P0 = n * kPcMap * kPcMap;
    using Im1 = NhwcIm2col<kPcC2, 4, 4, 2, kPcA1, kPcA1, kPcMap, kPcMap, 1>;  // dP2 windows per pcb pixel
    launch_wgrad6<32, 128, 1, 4>(pcb, 32, 32, Im2colT<Im1>{Im1{P2, P0}, 16 * kPcC2}, 16 * kPcC2, P0, w.slab,
                                 slab_floats(L), Gr + L.uw1, nullptr, st);
    colsum(P2, npix, kPcC2, w.colsum, Gr + L.ub1, st);
    DenseRows fb{P + L.uw1, 16 * kPcC2, 32};
    EpiMask ep{pcb, pcb, 32};
    launch_gemm_x6_sk<128, 32, 32, 4, 1>(Im1{P2, P0}, fb, ep, P0, 32, 16 * kPcC2, st, L);
  } else {
    // second layer: dW2 = A1^T x im2col(dP2) (block-diagonal mask), db2, dA1 masked in place, db1
    const int P1 = n * kPcA1 * kPcA1;
    using Im2 = NhwcIm2col<kPcC2, 4, 4, 2, kPcP, kPcP, kPcA1, kPcA1, 1>;  // dP2 windows per A1 pixel
    launch_wgrad6<64, 128, 2, 2>(A1, kPcC1, kPcC1, Im2colT<Im2>{Im2{P2, P1}, 16 * kPcC2}, 16 * kPcC2, P1, w.slab,
                                 slab_floats(L), Gr + L.uw2, nullptr, st);
    hipLaunchKernelGGL(pc_blockdiag_mask_kernel, dim3((kPcC1 * 16 * kPcC2 + 255) / 256), dim3(256), 0, st, Gr + L.uw2,
                       L.A);
    colsum(P2, npix, kPcC2, w.colsum, Gr + L.ub2, st);
    {
      DenseRows fb{P + L.uw2, 16 * kPcC2, kPcC1};
      EpiMask ep{A1, A1, kPcC1};
      launch_gemm_x6<64, 64, 32, 2, 2>(Im2{P2, P1}, fb, ep, P1, kPcC1, 16 * kPcC2, st);
    }
    colsum(A1, (int64_t)P1, kPcC1, w.colsum, Gr + L.ub1, st);
    // first layer: dW1[ci][tap][co] = sum pcb[iy][ix][ci] dA1[2iy + ky][2ix + kx][co]; dpcb =
    // conv(dA1, W1) under pc_base's ReLU, over pcb
    const int P0 = n * kPcMap * kPcMap;
    using Im1 = NhwcIm2col<kPcC1, 4, 4, 2, kPcA1, kPcA1, kPcMap, kPcMap, 1>;  // dA1 windows per pcb pixel
    launch_wgrad6<32, 128, 1, 4>(pcb, 32, 32, Im2colT<Im1>{Im1{A1, P0}, 16 * kPcC1}, 16 * kPcC1, P0, w.slab,
                                 slab_floats(L), Gr + L.uw1, nullptr, st);
    {
      DenseRows fb{P + L.uw1, 16 * kPcC1, 32};
      EpiMask ep{pcb, pcb, 32};
      // split-K below 128 tiles (the logged run's 4 envs: 54 tiles walking K = 1024: 40 us)
      launch_gemm_x6_sk<128, 32, 32, 4, 1>(Im1{A1, P0}, fb, ep, P0, 32, 16 * kPcC1, st, L);
    }
  }
  // pc_base: dW = dpcb^T x h (+ bias column), dh = dpcb x W
  {
    Im2colT<DenseRows> fbw{DenseRows{h, 512, n}, 512};
    launch_wgrad6<128, 128, 2, 2>(pcb, kPcBase, kPcBase, fbw, 512, n, w.slab, slab_floats(L), Gr + L.upw, Gr + L.upb,
                                  st);
  }
  tile_transpose(P + L.upw, kPcBase, 512, 512, w.wpct, kPcBase, st);
  {
    DenseRows fa{pcb, kPcBase, n};
    DenseRows fb{w.wpct, kPcBase, 512};
    EpiAcc ep{dh, 512, accumulate};
    launch_gemm_x6_sk<64, 64, 32, 2, 2>(fa, fb, ep, n, 512, kPcBase, st, L);
  }
  VN_HIP(hipGetLastError());
  return VN_OK;
}

// reward_prediction (goal.py:121-129): logits [n][4] (3 + pad) of x [n][3 FCIN] (three
// frames' conv_base maps, NHWC each; the rows of W are permuted to match).
int rp_forward_impl(const PolicyLayout& L, const float* P, const float* x, int n, float* out, hipStream_t st) {
  const int K = 3 * L.FCIN;
  DenseRows fa{x, K, n};
  DenseRows fb{P + L.urw, K, 3};
  EpiBiasAct ep{out, 4, P + L.urb, 0};
  launch_gemm_sk<64, 16, 32, 4, 1>(fa, fb, ep, n, 3, K, st, L);
  VN_HIP(hipGetLastError());
  return VN_OK;
}

int rp_backward_impl(const PolicyLayout& L, const float* P, const float* x, int n, const float* dout, float* Gr,
                     float* dx, float* slab, hipStream_t st) {
  const int K = 3 * L.FCIN;
  Im2colT<DenseRows> fbw{DenseRows{x, K, n}, K};
  launch_wgrad<32, 64, 2, 2>(dout, 4, 3, fbw, K, n, slab, slab_floats(L), Gr + L.urw, Gr + L.urb, st);
  if (dx) {
    const int64_t total = (int64_t)n * (K / 4);
    hipLaunchKernelGGL(rp_dx_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, dout, P + L.urw, n, K, dx);
  }
  VN_HIP(hipGetLastError());
  return VN_OK;
}

}  // namespace vn

using namespace vn;

struct vn_policy {
  PolicyLayout L;
};

namespace {
bool supported(int H, int W) {
  return (H == 84 && W == 84) || (H == 174 && W == 174) || (H == 300 && W == 400);
}

template <int H_, int W_>
struct GeoTag {
  static constexpr int H = H_, W = W_;
};

// Call f(GeoTag<H, W>{}) for the policy's frame geometry (the instantiated set).
template <class F>
int dispatch_geo(const PolicyLayout& L, F&& f) {
  if (L.H == 84 && L.W == 84) return f(GeoTag<84, 84>{});
  if (L.H == 174 && L.W == 174) return f(GeoTag<174, 174>{});
  if (L.H == 300 && L.W == 400) return f(GeoTag<300, 400>{});
  return fail(VN_EINVAL, "policy: unsupported frame geometry");
}

FrameSrc to_src(const vn_frames* f) {
  FrameSrc s{};
  s.base[0] = f->image;
  s.base[1] = f->goal;
  s.rows[0] = f->image_rows;
  s.rows[1] = f->goal_rows;
  s.stride = f->frame_bytes;
  s.f32[0] = f->image_f32;
  s.f32[1] = f->goal_f32;
  return s;
}
}  // namespace

extern "C" {

int vn_policy_create(int frame_h, int frame_w, int num_actions, vn_policy** out) {
  return vn_policy_create_ex(frame_h, frame_w, num_actions, 0, out);
}

int vn_policy_create_ex(int frame_h, int frame_w, int num_actions, int flags, vn_policy** out) {
  if (!out) return fail(VN_EINVAL, "vn_policy_create: out is NULL");
  if (flags & ~(VN_POLICY_LSTM | VN_POLICY_AUX | VN_POLICY_BIGHOUSE | VN_POLICY_UNREAL))
    return fail(VN_EINVAL, "vn_policy_create: unknown flags");
  if ((flags & VN_POLICY_BIGHOUSE) && (frame_h != 84 || frame_w != 84 || (flags & VN_POLICY_AUX)))
    return fail(VN_EINVAL, "vn_policy_create: BigHouseModel takes 84x84 frames (Linear(7*7*32)) and no aux heads");
  *out = nullptr;
  if (!supported(frame_h, frame_w))
    return fail(VN_EINVAL, "vn_policy_create: frame size must be 84x84, 174x174 or 300x400");
  if (num_actions < 1 || num_actions + 1 > OUT_LD) return fail(VN_EINVAL, "vn_policy_create: 1..7 actions");
  vn_policy* p = new (std::nothrow) vn_policy();
  if (!p) return fail(VN_ENOMEM, "vn_policy_create: host allocation");
  p->L = make_layout(frame_h, frame_w, num_actions, (flags & VN_POLICY_LSTM) ? 1 : 0, (flags & VN_POLICY_AUX) ? 1 : 0,
                     (flags & VN_POLICY_BIGHOUSE) ? 1 : 0, (flags & VN_POLICY_UNREAL) ? 1 : 0);
  // split-K scratch on the current device (16 MB; without it small batches run unsplit)
  p->L.sk = nullptr;
  p->L.sk_cap = 0;
  p->L.sk_dev = -1;
  constexpr int64_t kSplitKFloats = 4 << 20;
  if (hipGetDevice(&p->L.sk_dev) == hipSuccess && hipMalloc((void**)&p->L.sk, kSplitKFloats * 4) == hipSuccess) {
    p->L.sk_cap = kSplitKFloats;
  } else {
    p->L.sk = nullptr;
    (void)hipGetLastError();
  }
  *out = p;
  return VN_OK;
}

int vn_policy_destroy(vn_policy* p) {
  if (p && p->L.sk) (void)hipFree(p->L.sk);
  delete p;
  return VN_OK;
}

int vn_policy_info(vn_policy* p, int64_t* n_params, int64_t* act_floats_per_sample, int64_t* layout12) {
  if (!p) return fail(VN_EINVAL, "vn_policy_info: NULL policy");
  if (n_params) *n_params = p->L.n_params;
  if (act_floats_per_sample) {
    int64_t s = 0;
    for (int i = 0; i < 5; ++i) s += p->L.sz[i];
    *act_floats_per_sample = s + p->L.msz;
  }
  if (layout12)
    for (int i = 0; i < 6; ++i) {
      layout12[2 * i] = p->L.l[i].w;
      layout12[2 * i + 1] = p->L.l[i].b;
    }
  return VN_OK;
}

int vn_policy_workspace_floats(vn_policy* p, int64_t n, int64_t* floats) {
  if (!p || !floats || n <= 0) return fail(VN_EINVAL, "vn_policy_workspace_floats: bad args");
  *floats = workspace_floats(p->L, n);
  return VN_OK;
}

namespace {
int check_goal_runs(const vn_policy* p, const FrameSrc& src, int n, const vn_goal_runs* g, bool backward,
                    const char* who) {
  if (!g) return VN_OK;
  if (!goal_runs_ok(p->L, n) || src.f32[0] || src.f32[1])
    return fail(VN_EINVAL, std::string(who) + ": goal runs are not supported here (see vn_policy_goal_runs_supported)");
  if (!g->goal_list || !g->goal_count || !g->goal_delta)
    return fail(VN_EINVAL, std::string(who) + ": incomplete goal runs");
  if (backward && (!g->run_length || g->num_envs <= 0 || n % g->num_envs != 0))
    return fail(VN_EINVAL, std::string(who) + ": goal runs need run_length and num_envs dividing n");
  return VN_OK;
}
}  // namespace

int vn_policy_goal_runs_supported(vn_policy* p, int n, int* supported) {
  if (!p || !supported) return fail(VN_EINVAL, "vn_policy_goal_runs_supported: bad args");
  *supported = goal_runs_ok(p->L, n) ? 1 : 0;
  return VN_OK;
}

int vn_policy_forward(vn_policy* p, const float* params, const vn_frames* frames, int n, float* acts,
                      int64_t act_capacity, int64_t act_offset, float* out, vn_stream_t stream) {
  return vn_policy_forward_goals(p, params, frames, n, acts, act_capacity, act_offset, out, nullptr, stream);
}

int vn_policy_forward_goals(vn_policy* p, const float* params, const vn_frames* frames, int n, float* acts,
                            int64_t act_capacity, int64_t act_offset, float* out, const vn_goal_runs* goals,
                            vn_stream_t stream) {
  if (!p || !params || !frames || !acts || n <= 0) return fail(VN_EINVAL, "vn_policy_forward: bad args");
  if (!out && !p->L.lstm) return fail(VN_EINVAL, "vn_policy_forward: out is NULL");
  if (act_offset < 0 || act_offset + n > act_capacity)
    return fail(VN_EINVAL, "vn_policy_forward: samples exceed the activation capacity");
  const FrameSrc src = to_src(frames);
  if ((!src.base[0] && !src.f32[0]) || (!src.base[1] && !src.f32[1]))
    return fail(VN_EINVAL, "vn_policy_forward: missing frames");
  const int rc = check_goal_runs(p, src, n, goals, false, "vn_policy_forward");
  if (rc != VN_OK) return rc;
  const Acts a = acts_at(p->L, acts, act_capacity, act_offset);
  hipStream_t st = (hipStream_t)stream;
  if (p->L.arch == 1) return forward_bignet<84, 84>(p->L, params, src, n, a, out, st);
  return dispatch_geo(p->L, [&](auto g) {
    return forward_impl<decltype(g)::H, decltype(g)::W>(p->L, params, src, n, a, out, st, goals);
  });
}

int vn_policy_backward_ex(vn_policy* p, const float* params, const vn_frames* frames, int n, float* acts,
                          int64_t act_capacity, const float* dout, const float* dz5, const float* dx4_extra,
                          float* grads, float* workspace, vn_stream_t stream) {
  return vn_policy_backward_goals(p, params, frames, n, acts, act_capacity, dout, dz5, dx4_extra, grads, workspace,
                                  nullptr, stream);
}

int vn_policy_backward_goals(vn_policy* p, const float* params, const vn_frames* frames, int n, float* acts,
                             int64_t act_capacity, const float* dout, const float* dz5, const float* dx4_extra,
                             float* grads, float* workspace, const vn_goal_runs* goals, vn_stream_t stream) {
  if (!p || !params || !frames || !acts || !grads || !workspace || n <= 0 || (!dout && !dz5))
    return fail(VN_EINVAL, "vn_policy_backward: bad args");
  if (n > act_capacity) return fail(VN_EINVAL, "vn_policy_backward: n exceeds the activation capacity");
  const FrameSrc src = to_src(frames);
  const int rc = check_goal_runs(p, src, n, goals, true, "vn_policy_backward");
  if (rc != VN_OK) return rc;
  const Acts a = acts_at(p->L, acts, act_capacity, 0);
  const BwdWork w = carve(p->L, workspace, n);
  hipStream_t st = (hipStream_t)stream;
  const float* d = dz5 ? nullptr : dout;
  if (p->L.arch == 1) {
    // dx4_extra: dL/d conv_base's output (X3 here: reward prediction, bignet.py:98-103)
    return backward_bignet<84, 84>(p->L, params, src, n, a, d, dz5, dx4_extra, grads, w, st);
  }
  return dispatch_geo(p->L, [&](auto g) {
    return backward_impl<decltype(g)::H, decltype(g)::W>(p->L, params, src, n, a, d, dz5, dx4_extra, grads, w, st,
                                                         goals);
  });
}

int vn_policy_backward(vn_policy* p, const float* params, const vn_frames* frames, int n, float* acts,
                       int64_t act_capacity, const float* dout, float* grads, float* workspace,
                       vn_stream_t stream) {
  if (!dout) return fail(VN_EINVAL, "vn_policy_backward: dout is NULL");
  return vn_policy_backward_ex(p, params, frames, n, acts, act_capacity, dout, nullptr, nullptr, grads, workspace,
                               stream);
}

int vn_policy_backward_trunk(vn_policy* p, const float* params, const vn_frames* frames, int n, float* acts,
                             int64_t act_capacity, const float* dz5, float* grads, float* workspace,
                             vn_stream_t stream) {
  if (!dz5) return fail(VN_EINVAL, "vn_policy_backward_trunk: dz5 is NULL");
  return vn_policy_backward_ex(p, params, frames, n, acts, act_capacity, nullptr, dz5, nullptr, grads, workspace,
                               stream);
}

int vn_policy_unreal_info(vn_policy* p, int64_t* info8) {
  if (!p || !info8) return fail(VN_EINVAL, "vn_policy_unreal_info: bad args");
  if (!p->L.unreal) return fail(VN_EINVAL, "vn_policy_unreal_info: policy has no UNREAL heads");
  const PolicyLayout& L = p->L;
  const int64_t v[8] = {L.upw, L.upb, L.uw1, L.ub1, L.uw2, L.ub2, L.urw, L.urb};
  for (int i = 0; i < 8; ++i) info8[i] = v[i];
  return VN_OK;
}

int vn_pc_workspace_floats(vn_policy* p, int64_t* floats) {
  if (!p || !floats || !p->L.unreal) return fail(VN_EINVAL, "vn_pc_workspace_floats: bad args");
  *floats = pc_workspace_floats(p->L);
  return VN_OK;
}

int vn_pc_forward(vn_policy* p, const float* params, const float* h, int n, float* pcb, float* a1, float* p2, float* q,
                  float* workspace, vn_stream_t stream) {
  if (!p || !p->L.unreal || !params || !h || !pcb || (!a1 && p->L.arch != 1) || !p2 || !workspace || n <= 0)
    return fail(VN_EINVAL, "vn_pc_forward: bad args");
  return pc_forward_impl(p->L, params, h, n, pcb, a1, p2, q, pc_carve(p->L, workspace), (hipStream_t)stream);
}

int vn_pc_backward(vn_policy* p, const float* params, const float* h, int n, float* pcb, float* a1, float* p2,
                   const float* dq, float* grads, float* dh, int accumulate, float* workspace, vn_stream_t stream) {
  if (!p || !p->L.unreal || !params || !h || !pcb || (!a1 && p->L.arch != 1) || !p2 || !grads || !dh || !workspace ||
      n <= 0)
    return fail(VN_EINVAL, "vn_pc_backward: bad args");
  return pc_backward_impl(p->L, params, h, n, pcb, a1, p2, dq, grads, dh, accumulate, pc_carve(p->L, workspace),
                          (hipStream_t)stream);
}

int vn_rp_forward(vn_policy* p, const float* params, const float* x, int n, float* out, vn_stream_t stream) {
  if (!p || !p->L.unreal || !params || !x || !out || n <= 0) return fail(VN_EINVAL, "vn_rp_forward: bad args");
  return rp_forward_impl(p->L, params, x, n, out, (hipStream_t)stream);
}

int vn_rp_backward(vn_policy* p, const float* params, const float* x, int n, const float* dout, float* grads,
                   float* dx, float* workspace, vn_stream_t stream) {
  if (!p || !p->L.unreal || !params || !x || !dout || !grads || !workspace || n <= 0)
    return fail(VN_EINVAL, "vn_rp_backward: bad args");
  return rp_backward_impl(p->L, params, x, n, dout, grads, dx, pc_carve(p->L, workspace).slab, (hipStream_t)stream);
}

int vn_policy_aux_info(vn_policy* p, int64_t* info8) {
  if (!p || !info8) return fail(VN_EINVAL, "vn_policy_aux_info: bad args");
  if (!p->L.aux) return fail(VN_EINVAL, "vn_policy_aux_info: policy has no aux heads");
  const PolicyLayout& L = p->L;
  const int64_t v[8] = {L.aw1, L.ab1, L.aw2, L.ab2, L.AH, L.AW, L.PH, L.PW};
  for (int i = 0; i < 8; ++i) info8[i] = v[i];
  return VN_OK;
}

int vn_aux_workspace_floats(vn_policy* p, int64_t* floats) {
  if (!p || !floats || !p->L.aux) return fail(VN_EINVAL, "vn_aux_workspace_floats: bad args");
  *floats = aux_workspace_floats(p->L);
  return VN_OK;
}

int vn_aux_forward(vn_policy* p, const float* params, float* acts, int64_t act_capacity, int n, float* a1,
                   float* pred, float* workspace, vn_stream_t stream) {
  if (!p || !p->L.aux || !params || !acts || !a1 || !pred || !workspace || n <= 0 || n > act_capacity)
    return fail(VN_EINVAL, "vn_aux_forward: bad args");
  const Acts a = acts_at(p->L, acts, act_capacity, 0);
  const AuxWork w = aux_carve(p->L, workspace);
  hipStream_t st = (hipStream_t)stream;
  return dispatch_geo(p->L, [&](auto g) {
    return aux_forward_impl<decltype(g)::H, decltype(g)::W>(p->L, params, a.X[3], n, a1, pred, w, st);
  });
}

int vn_aux_target_table(vn_policy* p, const uint8_t* depth, const uint8_t* segmentation, int height, int width,
                        int64_t n_rows, float* table, vn_stream_t stream) {
  if (!p || !p->L.aux || !depth || !segmentation || !table || n_rows <= 0)
    return fail(VN_EINVAL, "vn_aux_target_table: bad args");
  const PolicyLayout& L = p->L;
  if (height < L.PH * kAuxCell || width < L.PW * kAuxCell)
    return fail(VN_EINVAL, "vn_aux_target_table: frames smaller than the crop");
  const int64_t total = n_rows * L.PH * L.PW;
  hipLaunchKernelGGL(aux_target_table_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, depth, segmentation, height, width, n_rows, L.PH, L.PW,
                     reinterpret_cast<f4*>(table));
  VN_HIP(hipGetLastError());
  return VN_OK;
}

int vn_aux_loss_grad(vn_policy* p, const float* pred, int n, const vn_aux_targets* targets, float weight,
                     float* dpred, float* stats4, vn_stream_t stream) {
  if (!p || !p->L.aux || !pred || !targets || !dpred || !stats4 || n <= 0 || !targets->table ||
      !targets->image_rows || !targets->goal_rows)
    return fail(VN_EINVAL, "vn_aux_loss_grad: bad args");
  const PolicyLayout& L = p->L;
  const int64_t total = (int64_t)n * L.PH * L.PW;
  const unsigned blocks = (unsigned)std::min<int64_t>(kAuxLossBlocks, (total + 255) / 256);
  hipLaunchKernelGGL(aux_loss_grad_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream,
                     n, L.PH, L.PW, pred, reinterpret_cast<const f4*>(targets->table), targets->image_rows,
                     targets->goal_rows, weight, dpred, stats4);
  VN_HIP(hipGetLastError());
  return VN_OK;
}

int vn_aux_forward_loss_grad(vn_policy* p, const float* params, float* acts, int64_t act_capacity, int n, float* a1,
                             float* pred, const vn_aux_targets* targets, float weight, float* dpred, float* stats4,
                             float* workspace, vn_stream_t stream) {
  if (!p || !p->L.aux || !params || !acts || !a1 || !pred || !targets || !targets->table || !targets->image_rows ||
      !targets->goal_rows || !dpred || !stats4 || !workspace || n <= 0 || n > act_capacity)
    return fail(VN_EINVAL, "vn_aux_forward_loss_grad: bad args");
  const Acts a = acts_at(p->L, acts, act_capacity, 0);
  const AuxWork w = aux_carve(p->L, workspace);
  return dispatch_geo(p->L, [&](auto g) {
    return aux_forward_loss_impl<decltype(g)::H, decltype(g)::W>(p->L, params, a.X[3], n, a1, pred, targets, weight,
                                                                  dpred, stats4, w, (hipStream_t)stream);
  });
}

int vn_aux_backward(vn_policy* p, const float* params, float* acts, int64_t act_capacity, int n, float* a1,
                    const float* dpred, float* grads, float* dx4, float* workspace, vn_stream_t stream) {
  if (!p || !p->L.aux || !params || !acts || !a1 || !dpred || !grads || !dx4 || !workspace || n <= 0 ||
      n > act_capacity)
    return fail(VN_EINVAL, "vn_aux_backward: bad args");
  const Acts a = acts_at(p->L, acts, act_capacity, 0);
  const AuxWork w = aux_carve(p->L, workspace);
  hipStream_t st = (hipStream_t)stream;
  return dispatch_geo(p->L, [&](auto g) {
    return aux_backward_impl<decltype(g)::H, decltype(g)::W>(p->L, params, a.X[3], n, a1, dpred, grads, dx4, w, st);
  });
}

int vn_policy_lstm_info(vn_policy* p, int64_t* info8) {
  if (!p || !info8) return fail(VN_EINVAL, "vn_policy_lstm_info: bad args");
  if (!p->L.lstm) return fail(VN_EINVAL, "vn_policy_lstm_info: policy has no recurrent core");
  const PolicyLayout& L = p->L;
  const int64_t v[8] = {L.lw, L.lbih, L.lbhh, L.xcat, L.xoff, L.lin, 512, 0};
  for (int i = 0; i < 8; ++i) info8[i] = v[i];
  return VN_OK;
}

int vn_lstm_workspace_floats(vn_policy* p, int T, int E, int64_t* floats) {
  if (!p || !floats || T <= 0 || E <= 0 || !p->L.lstm) return fail(VN_EINVAL, "vn_lstm_workspace_floats: bad args");
  *floats = lstm_workspace_floats(p->L, T, E);
  return VN_OK;
}

int vn_lstm_forward_step(vn_policy* p, const float* params, int E, const float* x5, const float* lra,
                         const float* mask, const float* h_prev, const float* c_prev, float* xcat, float* gates,
                         float* acts, float* c_out, float* h_out, vn_stream_t stream) {
  if (!p || !p->L.lstm || !params || E <= 0 || !x5 || !xcat || !gates || !acts || !c_out || !h_out)
    return fail(VN_EINVAL, "vn_lstm_forward_step: bad args");
  return lstm_forward_step(p->L, params, E, x5, lra, mask, h_prev, c_prev, xcat, gates, acts, c_out, h_out,
                           (hipStream_t)stream);
}

int vn_policy_heads(vn_policy* p, const float* params, const float* feat, int n, float* out, vn_stream_t stream) {
  if (!p || !params || !feat || !out || n <= 0) return fail(VN_EINVAL, "vn_policy_heads: bad args");
  return heads_forward(p->L, params, feat, n, out, (hipStream_t)stream);
}

int vn_lstm_backward(vn_policy* p, const float* params, int T, int E, const float* dout, const float* h_all,
                     const float* xcat_all, const float* acts_all, const float* c_all, const float* c_init,
                     const float* mask_all, const float* x5_all, float* dz5_all, float* grads, float* workspace,
                     vn_stream_t stream) {
  if (!p || !p->L.lstm || !params || T <= 0 || E <= 0 || !dout || !h_all || !xcat_all || !acts_all || !c_all ||
      !x5_all || !dz5_all || !grads || !workspace)
    return fail(VN_EINVAL, "vn_lstm_backward: bad args");
  if ((int64_t)T * E > (int64_t)1 << 30) return fail(VN_EINVAL, "vn_lstm_backward: T*E too large");
  const LstmWork w = lstm_carve(p->L, workspace, T, E);
  return lstm_backward(p->L, params, T, E, dout, h_all, xcat_all, acts_all, c_all, c_init, mask_all, x5_all, dz5_all,
                       grads, w, (hipStream_t)stream);
}

int vn_lstm_backward_ex(vn_policy* p, const float* params, int T, int E, const float* dout, const float* h_all,
                        const float* xcat_all, const float* acts_all, const float* c_all, const float* c_init,
                        const float* mask_all, const float* x5_all, const float* dh_extra, int extra_envs,
                        float* dz5_all, float* grads, float* workspace, vn_stream_t stream) {
  if (dh_extra && (extra_envs <= 0 || extra_envs > E))
    return fail(VN_EINVAL, "vn_lstm_backward_ex: extra_envs must be 1..E with dh_extra");
  if (!p || !p->L.lstm || !params || T <= 0 || E <= 0 || !dout || !h_all || !xcat_all || !acts_all || !c_all ||
      !x5_all || !dz5_all || !grads || !workspace)
    return fail(VN_EINVAL, "vn_lstm_backward_ex: bad args");
  if ((int64_t)T * E > (int64_t)1 << 30) return fail(VN_EINVAL, "vn_lstm_backward_ex: T*E too large");
  const LstmWork w = lstm_carve(p->L, workspace, T, E);
  return lstm_backward(p->L, params, T, E, dout, h_all, xcat_all, acts_all, c_all, c_init, mask_all, x5_all, dz5_all,
                       grads, w, (hipStream_t)stream, dh_extra, dh_extra ? extra_envs : 0);
}

}  // extern "C"
