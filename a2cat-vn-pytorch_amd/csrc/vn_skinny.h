// vn_skinny.h — products of a few rows on the fp32 VALU (included by vn_policy.hip).
//
// A rollout step of E envs runs its conv_merge, LSTM-gate and head products with M = E rows.
// For E <= kSkinnyRows the tensor-core tiles cannot fill the chip: the x6 path splits K into
// slabs and needs a second launch to reduce them and apply the epilogue, and each of those
// launches costs more than its arithmetic (the reference's own run is 4 envs). Here one
// workgroup computes kSkCols output columns of all M rows over the WHOLE K range — A staged
// in LDS chunk by chunk and read by every column group, B (weights, [N][K] k-contiguous) read
// once — with plain fp32 FMAs (the products are exact fp32 arithmetic like the x6 path, summed
// in another order), a 32-lane reduction, and the epilogue in the same launch. The LSTM step
// also folds in the xcat build and the cell (one launch instead of four), and the BPTT step
// its dh product and the next cell backward (one launch instead of three).
#pragma once

namespace vn {

constexpr int kSkinnyRows = 16;  // M at or below which the skinny path runs
constexpr int kSkCols = 8;       // output columns per workgroup: one 32-lane group each

template <class EP>
__device__ __forceinline__ void apply_epi(const EP& ep, int row, int col, float v) {
  if constexpr (has_pre_col<EP>::value)
    ep.post(row, col, v, ep.pre_col(col), 0);
  else if constexpr (has_pre_row<EP>::value)
    ep.post(row, col, v, ep.pre_row(row), 0);
  else if constexpr (has_pre<EP>::value)
    ep.post(row, col, v, ep.pre(row, col), 0);
  else
    ep(row, col, v, 0);
}

__device__ __forceinline__ float sum32(float v) {
#pragma unroll
  for (int o = 16; o > 0; o >>= 1) v += __shfl_xor(v, o, 32);
  return v;
}

// acc[m] (m < M) += this lane's share of sum_k A[m][k] B[k] over k < K. LPC lanes share a
// column (lane kl takes k = 4 kl + 4 LPC i of each chunk); A comes from fill(m, k) -> f4 (k % 4
// == 0, zeros past K), staged in As [MR][kc]; B is a 16-B aligned row. Per chunk of kc <= KB *
// 4 LPC values the lane's B loads are issued first, then the A loads of the chunk's staging,
// so both latencies are paid once (a chunk per memory round trip, not per 128 values). KB = the
// B f4 registers per lane, sized by the caller to the K it runs (a lane issues exactly KB loads
// per chunk: clamped, unconditional). All 256 threads of the workgroup call it (it
// synchronises).
constexpr int kSkKB = 24;  // B f4 registers per lane at most: chunks of up to 3072 values

template <int MR, int LPC, int KB>
constexpr int skinny_kc() {  // chunk length: KB * 4 LPC values, as the LDS allows (<= 128 KiB)
  return (MR * KB * 4 * LPC * 4 <= 128 * 1024) ? KB * 4 * LPC : (128 * 1024 / (MR * 4)) / (4 * LPC) * (4 * LPC);
}

struct RowsFill {  // dense rows A [M][lda] (16-B aligned, lda % 4 == 0)
  const float* A;
  int64_t lda;
  __device__ __forceinline__ f4 operator()(int m, int k) const {
    return *reinterpret_cast<const f4*>(A + (int64_t)m * lda + k);
  }
};

template <int MR, int LPC, int KB, class FILL>
__device__ __forceinline__ void skinny_dot(const FILL& fill, const float* __restrict__ B, int M, int K, float* As,
                                           float (&acc)[MR]) {
  constexpr int KC = skinny_kc<MR, LPC, KB>(), NB = KC / (4 * LPC);
  const int tid = threadIdx.x, kl = tid & (LPC - 1);
  // every load of a chunk (B, then all of A's staging from dense rows) is issued before the
  // first use: a staging loop that stored each value as it arrived paid one memory round trip
  // per 256 values (10 in a row for conv_merge's 4 x 2592)
  constexpr int NFI = (MR * KC / 4 + 255) / 256;  // staging f4 per thread, at most
  for (int k0 = 0; k0 < K; k0 += KC) {
    const int kc = min(KC, K - k0);
    f4 b[NB];
#pragma unroll
    for (int i = 0; i < NB; ++i)  // clamped (a lane past the chunk reloads its end; unused)
      b[i] = *reinterpret_cast<const f4*>(B + k0 + min(4 * kl + 4 * LPC * i, kc - 4));
    const int q4 = (kc + 3) / 4, nf = M * q4;
    if constexpr (std::is_same<FILL, RowsFill>::value) {
      f4 fr[NFI];
#pragma unroll
      for (int j = 0; j < NFI; ++j)
        if (j * 256 < nf) {  // wave-uniform
          const int i = min(tid + j * 256, nf - 1);
          const int m = i / q4, q = i - m * q4;
          fr[j] = fill(m, k0 + 4 * q);
        }
      __syncthreads();  // the previous chunk's reads are done
#pragma unroll
      for (int j = 0; j < NFI; ++j) {
        const int i = tid + j * 256;
        if (j * 256 < nf && i < nf) {
          const int m = i / q4, q = i - m * q4;
          *reinterpret_cast<f4*>(&As[m * KC + 4 * q]) = fr[j];
        }
      }
    } else {  // a gathering fill (the LSTM's xcat: three sources) measured faster value by value
      __syncthreads();
      for (int i = tid; i < nf; i += 256) {
        const int m = i / q4, q = i - m * q4;
        *reinterpret_cast<f4*>(&As[m * KC + 4 * q]) = fill(m, k0 + 4 * q);
      }
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const int kk = 4 * kl + 4 * LPC * i;
      if (kk < kc) {
#pragma unroll
        for (int m = 0; m < MR; ++m) {
          if (m < M) {
            const f4 a = *reinterpret_cast<const f4*>(&As[m * KC + kk]);
            float s = acc[m];
            s = fmaf(a[0], b[i][0], s);
            s = fmaf(a[1], b[i][1], s);
            s = fmaf(a[2], b[i][2], s);
            s = fmaf(a[3], b[i][3], s);
            acc[m] = s;
          }
        }
      }
    }
  }
  // the sum over the column's lanes within a wave (LPC = 128: each wave's half, combined by the caller)
#pragma unroll
  for (int m = 0; m < MR; ++m) {
    float v = acc[m];
#pragma unroll
    for (int o = (LPC < 64 ? LPC : 64) / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, LPC < 64 ? LPC : 64);
    acc[m] = v;
  }
}

// The f4 registers per lane for K at LPC lanes per column (one chunk when it fits kSkKB).
constexpr int skinny_kb(int K, int LPC) {
  return (K + 4 * LPC - 1) / (4 * LPC) < kSkKB ? (K + 4 * LPC - 1) / (4 * LPC) : kSkKB;
}

// C[m][col] = A[m] . B[col] for m < M <= MR, col < N; then the epilogue. 256 / LPC columns per
// workgroup: LPC = 32 (8 columns) for short rows, 128 (2 columns, two waves each, their sums
// added in wave order through LDS) where 8 columns per workgroup would leave most CUs idle
// (conv_merge: 512 columns -> 256 workgroups instead of 64, every weight byte streamed once).
template <int MR, int LPC, int KB, class EP>
__global__ __launch_bounds__(256) void skinny_kernel(const float* __restrict__ A, int64_t lda,
                                                     const float* __restrict__ B, int64_t ldb, EP ep, int M, int N,
                                                     int K) {
  __shared__ __attribute__((aligned(16))) float As[MR * skinny_kc<MR, LPC, KB>()];
  const int cg = threadIdx.x / LPC, kl = threadIdx.x & (LPC - 1);
  const int col = blockIdx.x * (256 / LPC) + cg;
  float acc[MR];
#pragma unroll
  for (int m = 0; m < MR; ++m) acc[m] = 0.0f;
  skinny_dot<MR, LPC, KB>(RowsFill{A, lda}, B + (int64_t)min(col, N - 1) * ldb, M, K, As, acc);
  if constexpr (LPC == 128) {
    __shared__ float red[2][MR];
    const int wave = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0 && (wave & 1)) {
#pragma unroll
      for (int m = 0; m < MR; ++m) red[wave >> 1][m] = acc[m];
    }
    __syncthreads();
    if ((threadIdx.x & 63) == 0 && !(wave & 1) && col < N) {
#pragma unroll
      for (int m = 0; m < MR; ++m)
        if (m < M) apply_epi(ep, m, col, acc[m] + red[wave >> 1][m]);
    }
  } else {
    if (kl == 0 && col < N) {
#pragma unroll
      for (int m = 0; m < MR; ++m)
        if (m < M) apply_epi(ep, m, col, acc[m]);
    }
  }
}

template <int MR, int LPC, class EP>
inline void launch_skinny_lpc(const float* A, int64_t lda, const float* B, int64_t ldb, EP ep, int M, int N, int K,
                              hipStream_t st) {
  const dim3 grid((N + 256 / LPC - 1) / (256 / LPC));
  // K-specific register counts: a lane issues exactly the loads its chunk uses
  if (K <= 4 * LPC * 4)
    hipLaunchKernelGGL((skinny_kernel<MR, LPC, 4, EP>), grid, dim3(256), 0, st, A, lda, B, ldb, ep, M, N, K);
  else if (K <= 4 * LPC * 8)
    hipLaunchKernelGGL((skinny_kernel<MR, LPC, 8, EP>), grid, dim3(256), 0, st, A, lda, B, ldb, ep, M, N, K);
  else
    hipLaunchKernelGGL((skinny_kernel<MR, LPC, (LPC == 128 ? 6 : kSkKB), EP>), grid, dim3(256), 0, st, A, lda, B, ldb,
                       ep, M, N, K);
}

template <class EP>
inline void launch_skinny(const float* A, int64_t lda, const float* B, int64_t ldb, EP ep, int M, int N, int K,
                          hipStream_t st) {
  if (N >= 256) {  // wide products (conv_merge): two columns per workgroup
    if (M <= 4)
      launch_skinny_lpc<4, 128>(A, lda, B, ldb, ep, M, N, K, st);
    else if (M <= 8)
      launch_skinny_lpc<8, 128>(A, lda, B, ldb, ep, M, N, K, st);
    else
      launch_skinny_lpc<kSkinnyRows, 128>(A, lda, B, ldb, ep, M, N, K, st);
  } else {
    if (M <= 4)
      launch_skinny_lpc<4, 32>(A, lda, B, ldb, ep, M, N, K, st);
    else if (M <= 8)
      launch_skinny_lpc<8, 32>(A, lda, B, ldb, ep, M, N, K, st);
    else
      launch_skinny_lpc<kSkinnyRows, 32>(A, lda, B, ldb, ep, M, N, K, st);
  }
}

// ---- conv3 + conv4 of a few envs, one launch ------------------------------------------
// conv3 (k4 s2 over the channel concat of the image and goal X2 maps, 64 channels) and the
// 1x1 conv4 (64 -> 32) are both local to an output pixel, so for a few envs one workgroup
// takes kC34Rows pixels through both: their im2col rows (kC34Rows x 1024) are gathered into
// LDS, thread (co, k sixteenth) sums 64 exact fp32 products per row against its W3 row
// segment (its 16 f4 of weights issued in one burst), the sixteen partials are added in a
// fixed order (+ bias, ReLU) into X3 (kept for the backward) and LDS, and the 32 conv4
// outputs of each pixel follow from there. Replaces the split-K conv3 product, its
// reduce/epilogue launch and the conv4 product (three launches per rollout step).
// k = (ky*4 + kx)*64 + g*32 + c as NhwcIm2col. Two pixels per workgroup: 4 envs' 324 pixels
// in 162 workgroups (1 / 2 / 4 / 8 pixels: 2.12 / 1.95 / 1.99 / 2.05 ms per 4-env update,
// profiles/r05/ab_c34/; the W3 rows a thread holds are read once per workgroup either way).
constexpr int kC34Rows = 2;

template <int H, int W, int OH, int OW, int R = kC34Rows>
__global__ __launch_bounds__(1024) void conv34_small_kernel(const float* __restrict__ X2, int M,
                                                            const float* __restrict__ W3, const float* __restrict__ b3,
                                                            const float* __restrict__ W4, const float* __restrict__ b4,
                                                            float* __restrict__ X3, float* __restrict__ X4) {
  __shared__ __attribute__((aligned(16))) float A[R][1024];
  __shared__ float part[16][R][64];
  __shared__ float x3s[R][64];
  __shared__ float w4s[32][65];  // W4, row stride 65: conv4's 32 lanes read distinct banks
  __shared__ float bs[96];       // b3 | b4
  const int tid = threadIdx.x, row0 = blockIdx.x * R;
  const int co = tid & 63, kq = tid >> 6;
  f4 wv[16];  // W3[co][64 kq .. 64 kq + 63]
  {
    const f4* w = reinterpret_cast<const f4*>(W3 + (int64_t)co * 1024 + kq * 64);
#pragma unroll
    for (int i = 0; i < 16; ++i) wv[i] = w[i];
  }
  // every global read is issued here, before the first barrier: one memory round trip
  for (int i = tid; i < 32 * 64; i += 1024) w4s[i >> 6][i & 63] = W4[i];
  if (tid < 96) bs[tid] = tid < 64 ? b3[tid] : b4[tid - 64];
#pragma unroll
  for (int i = tid; i < R * 256; i += 1024) {  // gather: f4 i of the block = (row, k / 4)
    const int r = i >> 8, k = (i & 255) * 4, m = min(row0 + r, M - 1);
    const int n = m / (OH * OW), rr = m - n * (OH * OW), oy = rr / OW, ox = rr - (rr / OW) * OW;
    const int c = k & 31, g = (k >> 5) & 1, t = k >> 6, ky = t >> 2, kx = t & 3;
    *reinterpret_cast<f4*>(&A[r][k]) =
        *reinterpret_cast<const f4*>(X2 + ((((int64_t)n * 2 + g) * H + oy * 2 + ky) * W + ox * 2 + kx) * 32 + c);
  }
  __syncthreads();
  {
    float acc[R];
#pragma unroll
    for (int r = 0; r < R; ++r) acc[r] = 0.0f;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const f4 a = *reinterpret_cast<const f4*>(&A[r][kq * 64 + 4 * i]);
        float s = acc[r];
        s = fmaf(a[0], wv[i][0], s);
        s = fmaf(a[1], wv[i][1], s);
        s = fmaf(a[2], wv[i][2], s);
        s = fmaf(a[3], wv[i][3], s);
        acc[r] = s;
      }
    }
#pragma unroll
    for (int r = 0; r < R; ++r) part[kq][r][co] = acc[r];
  }
  __syncthreads();
  if (tid < R * 64) {  // conv3 epilogue: (row, co), the 16 partials in a fixed order
    const int r = tid >> 6, c = tid & 63;
    float v = 0.0f;
#pragma unroll
    for (int q = 0; q < 16; ++q) v += part[q][r][c];
    v = fmaxf(v + bs[c], 0.0f);
    x3s[r][c] = v;
    if (row0 + r < M) X3[(int64_t)(row0 + r) * 64 + c] = v;
  }
  __syncthreads();
  if (tid < R * 32) {  // conv4: (row, co4)
    const int r = tid >> 5, c4 = tid & 31;
    float s = 0.0f;
#pragma unroll 8
    for (int k = 0; k < 64; ++k) s = fmaf(x3s[r][k], w4s[c4][k], s);
    if (row0 + r < M) X4[(int64_t)(row0 + r) * 32 + c4] = fmaxf(s + bs[64 + c4], 0.0f);
  }
}

// ---- LSTM step: xcat build + gates product + cell, one launch ----------------------
struct XcatFill {  // xcat_t[m] = [x5 (512) | lra (A+1) | 0 pad | m_t h_{t-1} (512)] (vn_lstm.h)
  const float* x5;
  const float* lra;
  const float* mask;
  const float* h_prev;
  int A1, xoff;
  __device__ __forceinline__ float at(int m, int k) const {
    if (k < 512) return x5[(int64_t)m * 512 + k];
    if (k < 512 + A1) return lra ? lra[(int64_t)m * A1 + (k - 512)] : 0.0f;
    if (k < xoff) return 0.0f;
    return h_prev ? h_prev[(int64_t)m * 512 + (k - xoff)] * (mask ? mask[m] : 1.0f) : 0.0f;
  }
  __device__ __forceinline__ f4 operator()(int m, int k) const {
    if (k + 3 < 512) return *reinterpret_cast<const f4*>(x5 + (int64_t)m * 512 + k);
    if (k >= xoff && h_prev && (xoff & 3) == 0) {
      const f4 h = *reinterpret_cast<const f4*>(h_prev + (int64_t)m * 512 + (k - xoff));
      const float mk = mask ? mask[m] : 1.0f;
      return f4{h[0] * mk, h[1] * mk, h[2] * mk, h[3] * mk};
    }
    return f4{at(m, k), at(m, k + 1), at(m, k + 2), at(m, k + 3)};
  }
};

// Workgroup b: hidden units 2b, 2b+1; column group cg = (gate cg >> 1, unit 2b + (cg & 1)).
template <int MR>
__global__ __launch_bounds__(256) void lstm_step_skinny_kernel(XcatFill xf, int E, int xcat,
                                                               const float* __restrict__ Wcat,
                                                               const float* __restrict__ bih,
                                                               const float* __restrict__ bhh,
                                                               const float* __restrict__ c_prev, float* xc_out,
                                                               float* acts, float* c_out, float* h_out) {
  constexpr int KB = 9;  // xcat = 512 + A + 1 padded + 512 <= 1152 (A <= 7): one chunk of 9 f4 per lane
  __shared__ __attribute__((aligned(16))) float As[MR * skinny_kc<MR, 32, KB>()];
  __shared__ float gs[MR][kSkCols];
  const int tid = threadIdx.x, cg = tid >> 5, kl = tid & 31;
  const int gate = cg >> 1, unit = 2 * blockIdx.x + (cg & 1), col = gate * 512 + unit;
  {  // this workgroup's slice of the xcat rows the backward keeps
    const int64_t total = (int64_t)E * xcat, per = (total + gridDim.x - 1) / gridDim.x;
    const int64_t lo = blockIdx.x * per, hi = min(total, lo + per);
    for (int64_t i = lo + tid; i < hi; i += 256) {
      const int m = (int)(i / xcat), k = (int)(i - (int64_t)m * xcat);
      xc_out[i] = xf.at(m, k);
    }
  }
  float acc[MR];
#pragma unroll
  for (int m = 0; m < MR; ++m) acc[m] = 0.0f;
  skinny_dot<MR, 32, KB>(xf, Wcat + (int64_t)col * xcat, E, xcat, As, acc);
  if (kl == 0) {
    const float b0 = bih[col], b1 = bhh[col];
#pragma unroll
    for (int m = 0; m < MR; ++m)
      if (m < E) gs[m][cg] = acc[m] + b0 + b1;  // EpiBias2's order
  }
  __syncthreads();
  if (tid < 2 * E) {  // the cell of (env m, unit): lstm_cell_kernel's arithmetic
    const int m = tid >> 1, u = tid & 1, j = 2 * blockIdx.x + u;
    const float mk = xf.mask ? xf.mask[m] : 1.0f;
    const float cp = c_prev ? c_prev[(int64_t)m * 512 + j] * mk : 0.0f;
    const float i = sigmoidf_(gs[m][0 + u]), f = sigmoidf_(gs[m][2 + u]), g = tanhf(gs[m][4 + u]),
                o = sigmoidf_(gs[m][6 + u]);
    const float c = f * cp + i * g;
    const float h = o * tanhf(c);
    float* a4 = acts + (int64_t)m * 2048;
    a4[j] = i;
    a4[512 + j] = f;
    a4[1024 + j] = g;
    a4[1536 + j] = o;
    c_out[(int64_t)m * 512 + j] = c;
    h_out[(int64_t)m * 512 + j] = h;
  }
}

// ---- BPTT step t: dh_{t-1} = m_t (dgates_t W_hh) and the cell backward of step t-1 --------
struct LstmBwdStep {
  const float* dgates_t;   // [E][2048] (read)
  const float* whh_t;      // W_hh^T rows: [512][2048] (row j = the weights of hidden input j)
  const float* mask_t;     // m_t [E] (may be NULL)
  const float* dh_heads;   // step t-1's [E][512]
  const float* dc_next;    // dc from step t's cell backward [E][512]
  const float* acts;       // step t-1's [E][2048]
  const float* c;          // c_{t-1} [E][512]
  const float* c_prev;     // c_{t-2} (or c_init) [E][512] (may be NULL)
  const float* mask_prev;  // m_{t-1} [E] (may be NULL)
  float* dgates_prev;      // step t-1's [E][2048] (out)
  float* dc_prev_out;      // [E][512] (out)
};

template <int MR>
__global__ __launch_bounds__(256) void lstm_bwd_skinny_kernel(LstmBwdStep p, int E) {
  constexpr int KB = 16;  // K = 2048: one chunk of 16 f4 per lane (MR = 16: two, as the LDS allows)
  __shared__ __attribute__((aligned(16))) float As[MR * skinny_kc<MR, 32, KB>()];
  const int cg = threadIdx.x >> 5, kl = threadIdx.x & 31;
  const int j = blockIdx.x * kSkCols + cg;
  float acc[MR];
#pragma unroll
  for (int m = 0; m < MR; ++m) acc[m] = 0.0f;
  skinny_dot<MR, 32, KB>(RowsFill{p.dgates_t, 2048}, p.whh_t + (int64_t)j * 2048, E, 2048, As, acc);
  if (kl < MR && kl < E) {  // lane m of the group: env m (lstm_cell_bwd_kernel's arithmetic)
    float v = 0.0f;
#pragma unroll
    for (int m = 0; m < MR; ++m)
      if (m == kl) v = acc[m];
    const int m = kl;
    const int64_t idx = (int64_t)m * 512 + j;
    const float dhn = v * (p.mask_t ? p.mask_t[m] : 1.0f);  // EpiLstmDh
    const float mk = p.mask_prev ? p.mask_prev[m] : 1.0f;
    const float* a4 = p.acts + (int64_t)m * 2048;
    const float i = a4[j], f = a4[512 + j], g = a4[1024 + j], o = a4[1536 + j];
    const float tc = tanhf(p.c[idx]);
    const float dh = p.dh_heads[idx] + dhn;
    const float dc = p.dc_next[idx] + dh * o * (1.0f - tc * tc);
    const float cp = p.c_prev ? p.c_prev[idx] * mk : 0.0f;
    float* d4 = p.dgates_prev + (int64_t)m * 2048;
    d4[j] = dc * g * i * (1.0f - i);
    d4[512 + j] = dc * cp * f * (1.0f - f);
    d4[1024 + j] = dc * i * (1.0f - g * g);
    d4[1536 + j] = dh * tc * o * (1.0f - o);
    p.dc_prev_out[idx] = dc * f * mk;
  }
}

}  // namespace vn
