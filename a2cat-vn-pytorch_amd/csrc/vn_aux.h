// vn_aux.h — AuxiliaryBigGoalHouseModel's deconv heads (models/goal.py:144-189) and the
// auxiliary deconv loss of experiments/ai2_auxiliary/trainer.py:9-55, included by
// vn_policy.hip after the GEMM launch helpers.
//
// Heads: three TimeDistributed(ConvTranspose2d(32,16,k4,s2), ReLU, ConvTranspose2d(16,C,k4,s2))
// on the conv_base map X4 [n][h3][w3][32] for depth (C=1), segmentation (3) and goal
// segmentation (3). The three first layers share their input and run as ONE deconv with 48
// output channels; the second layers run as one deconv 48 -> 8 whose weight is block
// diagonal (head h reads channels 16h..16h+15 and writes depth 0, mask 1-3, goal mask 4-6;
// channel 7 is padding), so its off-block gradient is masked to keep them structural zeros.
//
// A stride-2 k4 transposed conv is computed as the parity-class "dgrad" product of the
// trunk's backward (DgradA/DgradB loaders): out pixel (2yy+py, 2xx+px) sums the 2x2 input
// taps that reach it. Its backward is a plain stride-2 conv (NhwcIm2col) for the input
// gradient and a split-K wgrad for the weights. Weights are stored [Cin][ky][kx][Cout].
#pragma once

namespace vn {

constexpr int kAuxC1 = 48;  // 3 heads x 16
constexpr int kAuxC2 = 8;   // depth 1 + mask 3 + goal mask 3 + pad
constexpr int kAuxCell = 4; // deconv_cell_size = pc_cell_size (goal.py:70,148)

// Output pixel (2yy + PY, 2xx + PX) of a transposed conv, bias (+ ReLU), NHWC.
template <int OH, int OW, int PY, int PX, int HYC, int WXC>
struct EpiDeconv {
  float* Y;
  int C;
  const float* bias;
  int relu;
  __device__ __forceinline__ float pre_col(int col) const { return bias[col]; }
  __device__ __forceinline__ void post(int row, int col, float v, float b, int) const {
    constexpr int per = HYC * WXC;
    const int n = row / per;
    const int r = row - n * per;
    const int y = (r / WXC) * 2 + PY, x = (r % WXC) * 2 + PX;
    v += b;
    Y[(((int64_t)n * OH + y) * OW + x) * C + col] = relu ? fmaxf(v, 0.0f) : v;
  }
};

// dX masked by the ReLU that produced X, plus an extra gradient on the same tensor (the
// aux heads' gradient w.r.t. the conv_base map), both under the mask.
struct EpiMaskAdd {
  float* out;
  const float* X;
  int64_t ld;
  const float* extra;
  __device__ __forceinline__ float2 pre(int row, int col) const {
    const int64_t i = (int64_t)row * ld + col;
    return float2{X[i], extra[i]};
  }
  __device__ __forceinline__ void post(int row, int col, float v, float2 xe, int) const {
    out[(int64_t)row * ld + col] = xe.x > 0.0f ? v + xe.y : 0.0f;
  }
};

// Head of output channel c of the second layer (-1 = padding channel).
__device__ __forceinline__ int aux_head_of_out(int c) { return c == 0 ? 0 : (c <= 3 ? 1 : (c <= 6 ? 2 : -1)); }

// Zero the off-block entries of dW2 [48][16][8] (block-diagonal second layer).
__global__ void aux_blockdiag_mask_kernel(float* __restrict__ dW2) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= kAuxC1 * 16 * kAuxC2) return;
  const int ci = idx / (16 * kAuxC2), co = idx % kAuxC2;
  if (aux_head_of_out(co) != ci / 16) dW2[idx] = 0.0f;
}

// Column sums of src [rows][cols] (cols in {8, 16, 32, 48, 64}), deterministic: each
// thread owns 4 consecutive columns of a row group and streams 16-B loads down the rows;
// per-block partials are reduced in a fixed order.
__global__ __launch_bounds__(256) void colsum_partial_kernel(const float* __restrict__ src, int64_t rows, int cols,
                                                             float* __restrict__ partial) {
  __shared__ f4 sh[256];
  const int q = cols / 4;                 // float4 columns
  const int lanes = 256 / q;              // row lanes per block
  const int c4 = threadIdx.x % q, l = threadIdx.x / q;
  f4 s = f4zero();
  if (l < lanes)
    for (int64_t r = (int64_t)blockIdx.x * lanes + l; r < rows; r += (int64_t)gridDim.x * lanes)
      s += *reinterpret_cast<const f4*>(src + r * cols + c4 * 4);
  sh[threadIdx.x] = (l < lanes) ? s : f4zero();
  __syncthreads();
  if (threadIdx.x < q) {
    f4 t = f4zero();
    for (int j = 0; j < lanes; ++j) t += sh[j * q + threadIdx.x];
    *reinterpret_cast<f4*>(partial + (int64_t)blockIdx.x * cols + threadIdx.x * 4) = t;
  }
}

// One wave per column (grid = cols): lane l sums partials b = l (mod 64) in order, then a
// fixed xor tree (the one-thread-per-column form walked up to 512 dependent loads: ~100 us).
__global__ void colsum_final_kernel(const float* __restrict__ partial, int blocks, int cols, float* __restrict__ out) {
  const int c = blockIdx.x, l = threadIdx.x;
  float t = 0.0f;
  for (int b = l; b < blocks; b += 64) t += partial[(int64_t)b * cols + c];
  for (int o = 32; o > 0; o >>= 1) t += __shfl_xor(t, o);
  if (l == 0) out[c] = t;
}

// Per-state target table (built once per scene cache): for every arena row and prediction
// pixel, (depth, seg0, seg1, seg2) = avg_pool(centre crop(obs / 255), 4)
// (compute_auxiliary_target, trainer.py:9-15). The goal segmentation target of a sample is
// the seg part of its goal row's entry.
__global__ void aux_target_table_kernel(const uint8_t* __restrict__ depth, const uint8_t* __restrict__ seg, int H,
                                        int W, int64_t n_rows, int PH, int PW, f4* __restrict__ table) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= n_rows * PH * PW) return;
  const int64_t row = idx / (PH * PW);
  const int pix = (int)(idx - row * PH * PW);
  const int oy = pix / PW, ox = pix - (pix / PW) * PW;
  const int top = (H - PH * kAuxCell) / 2, left = (W - PW * kAuxCell) / 2;
  const int64_t HW = (int64_t)H * W;
  const uint8_t* d = depth + row * HW;
  const uint8_t* s = seg + row * HW * 3;
  float acc[4] = {0.0f, 0.0f, 0.0f, 0.0f};
  for (int dy = 0; dy < kAuxCell; ++dy) {
    const int64_t rp = (int64_t)(top + oy * kAuxCell + dy) * W + left + ox * kAuxCell;
    for (int dx = 0; dx < kAuxCell; ++dx) {
      acc[0] += (float)d[rp + dx];
      for (int c = 0; c < 3; ++c) acc[1 + c] += (float)s[(rp + dx) * 3 + c];
    }
  }
  constexpr float k = (1.0f / 255.0f) * (1.0f / (kAuxCell * kAuxCell));
  table[idx] = f4{acc[0] * k, acc[1] * k, acc[2] * k, acc[3] * k};
}

// Per-head MSE gradient against the table: dP = weight * 2 (P - target) / numel(head);
// stats[h] += sum (P - target)^2. Grid-stride over (sample, pixel): 2 x 16-B pred loads,
// 16-B target loads from the image row and the goal row, 2 x 16-B gradient stores; the
// statistics are reduced per workgroup (one atomic per workgroup and head).
constexpr int kAuxLossBlocks = 2048;

__global__ __launch_bounds__(256) void aux_loss_grad_kernel(int n, int PH, int PW, const float* __restrict__ P,
                                                            const f4* __restrict__ table,
                                                            const int32_t* __restrict__ img_rows,
                                                            const int32_t* __restrict__ goal_rows, float weight,
                                                            float* __restrict__ dP, float* __restrict__ stats) {
  __shared__ float red[3][4];
  float sq[3] = {0.0f, 0.0f, 0.0f};
  const int64_t total = (int64_t)n * PH * PW;
  const float inv[3] = {2.0f * weight / ((float)n * PH * PW), 2.0f * weight / (3.0f * n * PH * PW),
                        2.0f * weight / (3.0f * n * PH * PW)};
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int e = (int)(idx / (PH * PW));
    const int pix = (int)(idx - (int64_t)e * PH * PW);
    const f4 ti = table[(int64_t)img_rows[e] * PH * PW + pix];
    const f4 tg = table[(int64_t)goal_rows[e] * PH * PW + pix];
    const f4 p0 = *reinterpret_cast<const f4*>(P + idx * kAuxC2);
    const f4 p1 = *reinterpret_cast<const f4*>(P + idx * kAuxC2 + 4);
    const float pr[7] = {p0[0], p0[1], p0[2], p0[3], p1[0], p1[1], p1[2]};
    const float t[7] = {ti[0], ti[1], ti[2], ti[3], tg[1], tg[2], tg[3]};
    float g[8];
#pragma unroll
    for (int c = 0; c < 7; ++c) {
      const float d = pr[c] - t[c];
      const int h = c == 0 ? 0 : (c <= 3 ? 1 : 2);
      sq[h] += d * d;
      g[c] = d * inv[h];
    }
    g[7] = 0.0f;
    *reinterpret_cast<f4*>(dP + idx * kAuxC2) = f4{g[0], g[1], g[2], g[3]};
    *reinterpret_cast<f4*>(dP + idx * kAuxC2 + 4) = f4{g[4], g[5], g[6], g[7]};
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int h = 0; h < 3; ++h) {
    float v = sq[h];
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    if (lane == 0) red[h][wave] = v;
  }
  __syncthreads();
  if (threadIdx.x < 3) {
    const float v = red[threadIdx.x][0] + red[threadIdx.x][1] + red[threadIdx.x][2] + red[threadIdx.x][3];
    if (v != 0.0f) atomicAdd(stats + threadIdx.x, v);
  }
}

// Second head layer (48 -> 8 transposed conv, k4 s2, block-diagonal weights) as a direct
// kernel, optionally fused with the loss: SPI samples' A1 maps are staged in LDS (pixel
// stride 52 floats: 16 consecutive pixels on distinct bank quads, one zero pixel for the
// taps outside the map). Each pair of waves owns one parity class (py, px), so the weights
// of its taps are wave-uniform, and a lane computes FOUR output pixels of its class along x,
// (2yy + py, 2(xb + i XB) + px), i = 0..3: every weight it reads feeds 4 pixels (the
// one-pixel form read 4 broadcast weight vectors per 16-B A1 read and was bound by LDS
// reads). The four are XB apart so that consecutive lanes read consecutive A1 pixels (the
// pixel stride 52 puts 16 of them on distinct bank quads; 4 adjacent pixels per lane put
// lanes 4 pixels apart: 4-way conflicts, 56 % of the LDS cycles). Each output sums the 2x2 taps that reach it over only its
// head's own 16 input channels (4 x (16 + 48 + 48) = 448 FMAs per pixel; the GEMM form
// multiplied the 2/3 structural zeros and padded N = 8 to 16), in the same order as before
// (bit-identical): 174x174 7.74 -> 6.74 ms per update. The weights stay in LDS
// [cls][tap][ci][8]; scalar loads from the constant address space measured 7.35 ms.
// !LOSS: writes pred [n][PH][PW][8]. LOSS: the per-head MSE gradient against the target
// table goes straight to dpred (pred is never written) and the squared errors to
// stats[0..2] (aux_loss_grad_kernel's contract).
constexpr int kAux2Threads = 512;
constexpr int kAux2Pst = 52;
constexpr int kAux2Px = 4;  // output pixels per lane

template <int AH, int AW>
constexpr int aux2_spi() {
  constexpr int per = (AH * AW + 1) * kAux2Pst * 4;
  return per * 2 <= 96 * 1024 ? (96 * 1024 / per < 8 ? 96 * 1024 / per : 8) : 1;
}
constexpr int kAux2Wfl = 4 * 4 * kAuxC1 * kAuxC2;  // weights [class][tap][ci][8] in LDS
template <int AH, int AW>
constexpr size_t aux2_lds() {
  return (size_t)aux2_spi<AH, AW>() * (AH * AW + 1) * kAux2Pst * 4 + kAux2Wfl * 4;
}
template <int AH, int AW>
constexpr bool aux2_fits() {
  return aux2_lds<AH, AW>() <= 160 * 1024;
}

template <int AH, int AW, int PH, int PW, bool LOSS>
__global__ __launch_bounds__(kAux2Threads) void aux_deconv2_kernel(const float* __restrict__ A1, int n,
                                                                    const float* __restrict__ W2,
                                                                    const float* __restrict__ b2,
                                                                    float* __restrict__ pred,
                                                                    const f4* __restrict__ table,
                                                                    const int32_t* __restrict__ img_rows,
                                                                    const int32_t* __restrict__ goal_rows,
                                                                    float weight, float* __restrict__ dpred,
                                                                    float* __restrict__ stats) {
  constexpr int SPI = aux2_spi<AH, AW>();
  constexpr int NPX = AH * AW, SST = (NPX + 1) * kAux2Pst;  // pixels, per-sample LDS stride
  constexpr int HYC = PH / 2, WXC = PW / 2;                 // output pixels per class: HYC x WXC
  constexpr int XB = (WXC + kAux2Px - 1) / kAux2Px, RT = HYC * XB;  // lane tasks per class and sample
  static_assert(PH == 2 * AH + 2 && PW == 2 * AW + 2, "k4 s2 transposed conv geometry");
  static_assert(kAux2Threads == 512, "two waves per parity class");
  extern __shared__ __attribute__((aligned(16))) float as_aux[];
  float* ws_aux = as_aux + SPI * SST;  // [cls][tap = 2a + b][ci][8]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int cls = __builtin_amdgcn_readfirstlane(wave >> 1), py = cls >> 1, px = cls & 1;
  for (int i = tid; i < SPI * 48; i += kAux2Threads) as_aux[(i / 48) * SST + NPX * kAux2Pst + i % 48] = 0.0f;
  for (int i = tid; i < kAux2Wfl; i += kAux2Threads) {
    const int c = i & 7, ci = (i >> 3) % kAuxC1, tap = (i / (8 * kAuxC1)) & 3, cl = i / (32 * kAuxC1);
    const int ky = (cl >> 1) + 2 * (tap >> 1), kx = (cl & 1) + 2 * (tap & 1);
    ws_aux[i] = W2[(ci * 4 + ky) * 32 + kx * 8 + c];
  }
  float bias[7];
#pragma unroll
  for (int c = 0; c < 7; ++c) bias[c] = b2[c];
#pragma unroll
  for (int c = 0; c < 7; ++c) asm volatile("" ::"v"(bias[c]));  // landed before the item loop's prefetches
  const float inv[3] = {2.0f * weight / ((float)n * PH * PW), 2.0f * weight / (3.0f * n * PH * PW),
                        2.0f * weight / (3.0f * n * PH * PW)};
  float sq[3] = {0.0f, 0.0f, 0.0f};
  // the next item's A1 maps are loaded into registers while this one computes
  constexpr int NV = (SPI * NPX * 12 + kAux2Threads - 1) / kAux2Threads;
  f4 pre[NV];
  auto load_item = [&](int s0) {
    const int nv = min(SPI, n - s0) * NPX * 12;
    const f4* src = reinterpret_cast<const f4*>(A1 + (int64_t)s0 * NPX * 48);
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      const int i = tid + j * kAux2Threads;
      if (i < nv) pre[j] = src[i];
    }
  };
  if ((int)blockIdx.x * SPI < n) load_item(blockIdx.x * SPI);
  for (int s0 = blockIdx.x * SPI; s0 < n; s0 += gridDim.x * SPI) {
    const int ns = min(SPI, n - s0);
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      const int i = tid + j * kAux2Threads;
      if (i < ns * NPX * 12) {
        const int sp = i / (NPX * 12), r = i - sp * (NPX * 12), pxl = r / 12, c4 = r - (r / 12) * 12;
        *reinterpret_cast<f4*>(as_aux + sp * SST + pxl * kAux2Pst + 4 * c4) = pre[j];
      }
    }
    __syncthreads();
    if (s0 + (int)gridDim.x * SPI < n) load_item(s0 + gridDim.x * SPI);
    for (int t = (wave & 1) * 64 + lane; t < ns * RT; t += 128) {
      const int sp = t / RT, r = t - sp * RT, yy = r / XB, xb = r - (r / XB) * XB, s = s0 + sp;
      const int npx = (WXC - xb + XB - 1) / XB;  // pixels xb + i XB < WXC
      // targets issued before the products. The goal's depth (tg .x) is not a target: loading
      // the whole f4 let the register allocator reuse that dead lane right away, which forced an
      // s_waitcnt vmcnt(0) on all eight loads before the products (round 6); only .yzw is loaded
      f4 ti[kAux2Px];
      float tg[kAux2Px][4];
      if constexpr (LOSS) {
        const int64_t ib = (int64_t)img_rows[s] * PH * PW, gb = (int64_t)goal_rows[s] * PH * PW;
#pragma unroll
        for (int i = 0; i < kAux2Px; ++i) {
          const int pix = (2 * yy + py) * PW + 2 * min(xb + i * XB, WXC - 1) + px;
          ti[i] = table[ib + pix];
          {
            const float* g3 = reinterpret_cast<const float*>(table + gb + pix) + 1;
            tg[i][1] = g3[0];
            tg[i][2] = g3[1];
            tg[i][3] = g3[2];
          }
        }
      }
      float o[kAux2Px][7];
#pragma unroll
      for (int i = 0; i < kAux2Px; ++i)
#pragma unroll
        for (int c = 0; c < 7; ++c) o[i][c] = bias[c];
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) {
          const int iy = yy - a;
          const float* ap[kAux2Px];
#pragma unroll
          for (int i = 0; i < kAux2Px; ++i) {
            const int ix = xb + i * XB - b;
            const bool ok = iy >= 0 && iy < AH && ix >= 0 && ix < AW;
            ap[i] = as_aux + sp * SST + (ok ? iy * AW + ix : NPX) * kAux2Pst;
          }
          const float* wl = ws_aux + ((cls * 4 + 2 * a + b) * kAuxC1) * 8;
#pragma unroll
          for (int hd = 0; hd < 3; ++hd)  // head hd reads input channels 16hd .. 16hd + 15
#pragma unroll 2
            for (int kq = 0; kq < 4; ++kq) {
              const int k = 4 * hd + kq;
              f4 av[kAux2Px];
#pragma unroll
              for (int i = 0; i < kAux2Px; ++i) av[i] = *reinterpret_cast<const f4*>(ap[i] + 4 * k);
#pragma unroll
              for (int jj = 0; jj < 4; ++jj) {
                const int ci = 4 * k + jj;
                const f4 wv = reinterpret_cast<const f4*>(wl + ci * 8)[hd < 2 ? 0 : 1];
#pragma unroll
                for (int i = 0; i < kAux2Px; ++i) {
                  if (hd == 0) {
                    o[i][0] = fmaf(av[i][jj], wv[0], o[i][0]);
                  } else if (hd == 1) {
                    o[i][1] = fmaf(av[i][jj], wv[1], o[i][1]);
                    o[i][2] = fmaf(av[i][jj], wv[2], o[i][2]);
                    o[i][3] = fmaf(av[i][jj], wv[3], o[i][3]);
                  } else {
                    o[i][4] = fmaf(av[i][jj], wv[0], o[i][4]);
                    o[i][5] = fmaf(av[i][jj], wv[1], o[i][5]);
                    o[i][6] = fmaf(av[i][jj], wv[2], o[i][6]);
                  }
                }
              }
            }
        }
#pragma unroll
      for (int i = 0; i < kAux2Px; ++i) {
        if (i >= npx) break;
        const int64_t pix = (int64_t)s * PH * PW + (2 * yy + py) * PW + 2 * (xb + i * XB) + px;
        if constexpr (!LOSS) {
          *reinterpret_cast<f4*>(pred + pix * kAuxC2) = f4{o[i][0], o[i][1], o[i][2], o[i][3]};
          *reinterpret_cast<f4*>(pred + pix * kAuxC2 + 4) = f4{o[i][4], o[i][5], o[i][6], 0.0f};
        } else {
          const float tv[7] = {ti[i][0], ti[i][1], ti[i][2], ti[i][3], tg[i][1], tg[i][2], tg[i][3]};
          float g[8];
#pragma unroll
          for (int c = 0; c < 7; ++c) {
            const float d = o[i][c] - tv[c];
            const int h = c == 0 ? 0 : (c <= 3 ? 1 : 2);
            sq[h] += d * d;
            g[c] = d * inv[h];
          }
          g[7] = 0.0f;
          *reinterpret_cast<f4*>(dpred + pix * kAuxC2) = f4{g[0], g[1], g[2], g[3]};
          *reinterpret_cast<f4*>(dpred + pix * kAuxC2 + 4) = f4{g[4], g[5], g[6], g[7]};
        }
      }
    }
    __syncthreads();
  }
  if constexpr (LOSS) {  // per-workgroup statistics (the staging area is free after the last barrier)
    float* red = as_aux;   // [3][waves]
    constexpr int NWV = kAux2Threads / 64;
    const int lane = tid & 63, wave = tid >> 6;
#pragma unroll
    for (int h = 0; h < 3; ++h) {
      float v = sq[h];
      for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
      if (lane == 0) red[h * NWV + wave] = v;
    }
    __syncthreads();
    if (tid < 3) {
      float v = 0.0f;
      for (int w = 0; w < NWV; ++w) v += red[tid * NWV + w];
      if (v != 0.0f) atomicAdd(stats + tid, v);
    }
  }
}

// The same second layer for maps whose A1 does not fit the LDS (300x400: 36x48x48 floats per
// sample): work item = (sample, band of BYC class rows yy), staging the BYC + 1 A1 rows its taps
// read (rows yy - 1 .. yy + BYC - 1; rows outside the map read the zero pixel). Same lane
// tasks (four output pixels XB apart), same sums in the same order (bit-identical to the
// whole-map form), the next item's rows prefetched into registers.
constexpr size_t aux2b_lds(int aw, int byc) { return (size_t)((byc + 1) * aw + 1) * kAux2Pst * 4 + kAux2Wfl * 4; }
// class rows per band: the lane tasks of a band fit one pass of a wave pair (BYC x XB <= 128)
// and the staged rows fit the LDS; 0 = no banded form
template <int AW, int PW>
constexpr int aux2_byc() {
  constexpr int XB = (PW / 2 + kAux2Px - 1) / kAux2Px;
  int b = 128 / XB;
  // and the prefetch registers of a band's rows stay within the whole-map kernel's (11 f4)
  while (b > 0 && (aux2b_lds(AW, b) > 150 * 1024 || ((b + 1) * AW * 12 + kAux2Threads - 1) / kAux2Threads > 11)) --b;
  return b;
}

template <int AH, int AW, int PH, int PW, bool LOSS, int BYC>
__global__ __launch_bounds__(kAux2Threads) void aux_deconv2_band_kernel(const float* __restrict__ A1, int n,
                                                                         const float* __restrict__ W2,
                                                                         const float* __restrict__ b2,
                                                                         float* __restrict__ pred,
                                                                         const f4* __restrict__ table,
                                                                         const int32_t* __restrict__ img_rows,
                                                                         const int32_t* __restrict__ goal_rows,
                                                                         float weight, float* __restrict__ dpred,
                                                                         float* __restrict__ stats) {
  constexpr int NR = BYC + 1, NPX = NR * AW;                // staged rows, pixels (+ one zero pixel)
  constexpr int HYC = PH / 2, WXC = PW / 2;
  constexpr int NBAND = (HYC + BYC - 1) / BYC;
  constexpr int XB = (WXC + kAux2Px - 1) / kAux2Px, RT = BYC * XB;
  static_assert(PH == 2 * AH + 2 && PW == 2 * AW + 2, "k4 s2 transposed conv geometry");
  extern __shared__ __attribute__((aligned(16))) float as_auxb[];
  float* ws_aux = as_auxb + (NPX + 1) * kAux2Pst;  // [cls][tap = 2a + b][ci][8]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int cls = __builtin_amdgcn_readfirstlane(wave >> 1), py = cls >> 1, px = cls & 1;
  for (int i = tid; i < 48; i += kAux2Threads) as_auxb[NPX * kAux2Pst + i] = 0.0f;
  for (int i = tid; i < kAux2Wfl; i += kAux2Threads) {
    const int c = i & 7, ci = (i >> 3) % kAuxC1, tap = (i / (8 * kAuxC1)) & 3, cl = i / (32 * kAuxC1);
    const int ky = (cl >> 1) + 2 * (tap >> 1), kx = (cl & 1) + 2 * (tap & 1);
    ws_aux[i] = W2[(ci * 4 + ky) * 32 + kx * 8 + c];
  }
  float bias[7];
#pragma unroll
  for (int c = 0; c < 7; ++c) bias[c] = b2[c];
#pragma unroll
  for (int c = 0; c < 7; ++c) asm volatile("" ::"v"(bias[c]));
  const float inv[3] = {2.0f * weight / ((float)n * PH * PW), 2.0f * weight / (3.0f * n * PH * PW),
                        2.0f * weight / (3.0f * n * PH * PW)};
  float sq[3] = {0.0f, 0.0f, 0.0f};
  constexpr int NV = (NPX * 12 + kAux2Threads - 1) / kAux2Threads;
  f4 pre[NV];
  // rows y0 - 1 .. y0 + BYC - 1 of sample s; rows outside the map load row 0 and stage zeros
  auto load_item = [&](int it) {
    const int s = it / NBAND, y0 = (it - (it / NBAND) * NBAND) * BYC;
    const f4* src = reinterpret_cast<const f4*>(A1 + (int64_t)s * AH * AW * kAuxC1);
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      const int i = min(tid + j * kAux2Threads, NPX * 12 - 1);
      const int r = i / (AW * 12), rem = i - r * (AW * 12);
      const int iy = y0 - 1 + r;
      const f4 v = src[(int64_t)(iy >= 0 && iy < AH ? iy : 0) * AW * 12 + rem];
      pre[j] = (iy >= 0 && iy < AH) ? v : f4{0.f, 0.f, 0.f, 0.f};
    }
  };
  const int n_items = n * NBAND;
  if ((int)blockIdx.x < n_items) load_item(blockIdx.x);
  for (int it = blockIdx.x; it < n_items; it += gridDim.x) {
    const int s = it / NBAND, y0 = (it - (it / NBAND) * NBAND) * BYC;
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      const int i = tid + j * kAux2Threads;
      if (i < NPX * 12) {
        const int pxl = i / 12, c4 = i - (i / 12) * 12;
        *reinterpret_cast<f4*>(as_auxb + pxl * kAux2Pst + 4 * c4) = pre[j];
      }
    }
    __syncthreads();
    if (it + (int)gridDim.x < n_items) load_item(it + gridDim.x);
    for (int t = (wave & 1) * 64 + lane; t < RT; t += 128) {
      const int yl = t / XB, xb = t - (t / XB) * XB, yy = y0 + yl;
      if (yy >= HYC) continue;  // the last band's rows past the map
      const int npx = (WXC - xb + XB - 1) / XB;
      f4 ti[kAux2Px];
      float tg[kAux2Px][4];  // .yzw only (see aux_deconv2_kernel)
      if constexpr (LOSS) {
        const int64_t ib = (int64_t)img_rows[s] * PH * PW, gb = (int64_t)goal_rows[s] * PH * PW;
#pragma unroll
        for (int i = 0; i < kAux2Px; ++i) {
          const int pix = (2 * yy + py) * PW + 2 * min(xb + i * XB, WXC - 1) + px;
          ti[i] = table[ib + pix];
          {
            const float* g3 = reinterpret_cast<const float*>(table + gb + pix) + 1;
            tg[i][1] = g3[0];
            tg[i][2] = g3[1];
            tg[i][3] = g3[2];
          }
        }
      }
      float o[kAux2Px][7];
#pragma unroll
      for (int i = 0; i < kAux2Px; ++i)
#pragma unroll
        for (int c = 0; c < 7; ++c) o[i][c] = bias[c];
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) {
          const int iy = yy - a, rl = yl + 1 - a;  // staged row of iy
          const float* ap[kAux2Px];
#pragma unroll
          for (int i = 0; i < kAux2Px; ++i) {
            const int ix = xb + i * XB - b;
            const bool ok = iy >= 0 && iy < AH && ix >= 0 && ix < AW;
            ap[i] = as_auxb + (ok ? rl * AW + ix : NPX) * kAux2Pst;
          }
          const float* wl = ws_aux + ((cls * 4 + 2 * a + b) * kAuxC1) * 8;
#pragma unroll
          for (int hd = 0; hd < 3; ++hd)
#pragma unroll 2
            for (int kq = 0; kq < 4; ++kq) {
              const int k = 4 * hd + kq;
              f4 av[kAux2Px];
#pragma unroll
              for (int i = 0; i < kAux2Px; ++i) av[i] = *reinterpret_cast<const f4*>(ap[i] + 4 * k);
#pragma unroll
              for (int jj = 0; jj < 4; ++jj) {
                const int ci = 4 * k + jj;
                const f4 wv = reinterpret_cast<const f4*>(wl + ci * 8)[hd < 2 ? 0 : 1];
#pragma unroll
                for (int i = 0; i < kAux2Px; ++i) {
                  if (hd == 0) {
                    o[i][0] = fmaf(av[i][jj], wv[0], o[i][0]);
                  } else if (hd == 1) {
                    o[i][1] = fmaf(av[i][jj], wv[1], o[i][1]);
                    o[i][2] = fmaf(av[i][jj], wv[2], o[i][2]);
                    o[i][3] = fmaf(av[i][jj], wv[3], o[i][3]);
                  } else {
                    o[i][4] = fmaf(av[i][jj], wv[0], o[i][4]);
                    o[i][5] = fmaf(av[i][jj], wv[1], o[i][5]);
                    o[i][6] = fmaf(av[i][jj], wv[2], o[i][6]);
                  }
                }
              }
            }
        }
#pragma unroll
      for (int i = 0; i < kAux2Px; ++i) {
        if (i >= npx) break;
        const int64_t pix = (int64_t)s * PH * PW + (2 * yy + py) * PW + 2 * (xb + i * XB) + px;
        if constexpr (!LOSS) {
          *reinterpret_cast<f4*>(pred + pix * kAuxC2) = f4{o[i][0], o[i][1], o[i][2], o[i][3]};
          *reinterpret_cast<f4*>(pred + pix * kAuxC2 + 4) = f4{o[i][4], o[i][5], o[i][6], 0.0f};
        } else {
          const float tv[7] = {ti[i][0], ti[i][1], ti[i][2], ti[i][3], tg[i][1], tg[i][2], tg[i][3]};
          float g[8];
#pragma unroll
          for (int c = 0; c < 7; ++c) {
            const float d = o[i][c] - tv[c];
            const int h = c == 0 ? 0 : (c <= 3 ? 1 : 2);
            sq[h] += d * d;
            g[c] = d * inv[h];
          }
          g[7] = 0.0f;
          *reinterpret_cast<f4*>(dpred + pix * kAuxC2) = f4{g[0], g[1], g[2], g[3]};
          *reinterpret_cast<f4*>(dpred + pix * kAuxC2 + 4) = f4{g[4], g[5], g[6], g[7]};
        }
      }
    }
    __syncthreads();
  }
  if constexpr (LOSS) {
    float* red = as_auxb;
    constexpr int NWV = kAux2Threads / 64;
#pragma unroll
    for (int h = 0; h < 3; ++h) {
      float v = sq[h];
      for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
      if (lane == 0) red[h * NWV + wave] = v;
    }
    __syncthreads();
    if (tid < 3) {
      float v = 0.0f;
      for (int w = 0; w < NWV; ++w) v += red[tid * NWV + w];
      if (v != 0.0f) atomicAdd(stats + tid, v);
    }
  }
}

// ---- fused second-layer backward ------------------------------------------------------
// One pass over (A1, dP) per sample replaces four launches (dW2 product, dA1 product with
// its ReLU mask, and the two bias column sums), and keeps the block-diagonal structure the
// GEMM forms multiplied as zeros: head h's 16 input channels only meet its own output
// channels (1, 3, 3), so dW2 has 16 x 16 x 7 live entries (of 48 x 128) and dA1 a K of
// 16 x nco per head. Work per workgroup: one sample at a time, its dP map staged in LDS
// (pixel stride 9 floats: 16 pixels two apart land on distinct banks); each wave takes
// 16-pixel tiles of the A1 map and runs, on v_mfma_f32_16x16x4f32,
//   dW2 (per head, C[ci][tap,co] += A1[px][ci] * dP[2y+ky][2x+kx][co] over the tile's 16
//        pixels; 7 accumulator tiles held across all the workgroup's samples), and
//   dA1 (C[px][ci] = sum_{tap,co} dP[2y+ky][2x+kx][co] * W2[ci][tap][co], weights in
//        registers), masked by A1 > 0 and written over A1 in place (the tile's A1 is read
//        by the same wave before it is overwritten);
// db1 (column sums of dA1) and db2 (of dP) ride along. Per-workgroup partials
// [7][4][64] + 48 + 8 are reduced in a fixed order (deterministic) by the finish kernel.
constexpr int kAuxBThreads = 512;
constexpr int kAuxBDs = 9;                                  // LDS floats per dP pixel
constexpr int kAuxBPart = 7 * 4 * 64 + kAuxC1 + kAuxC2;     // floats per workgroup partial
template <int PH, int PW>
constexpr size_t auxb_lds() {
  return (size_t)PH * PW * kAuxBDs * 4;
}
template <int AH, int AW, int PH, int PW>
constexpr bool auxb_fits() {
  return (AH * AW) % 16 == 0 && auxb_lds<PH, PW>() <= 80 * 1024 && auxb_lds<PH, PW>() >= 7 * 4 * 64 * 4 + 64 * 4;
}
// Maps whose dP does not fit (300x400: 74x98x8) run in bands of BYA A1 rows over the 2 BYA + 2
// dP rows under them: the largest BYA whose staged rows fit 80 KB with tiles (16 A1 pixels)
// spread evenly over the 8 waves (0 = no banded form).
constexpr size_t auxb_band_lds(int pw, int bya) { return (size_t)(2 * bya + 2) * pw * kAuxBDs * 4; }
template <int AH, int AW, int PH, int PW>
constexpr int auxb_bya() {
  for (int b = AH; b >= 1; --b)
    if ((b * AW) % 128 == 0 && auxb_band_lds(PW, b) <= 80 * 1024 && auxb_band_lds(PW, b) >= 7 * 4 * 64 * 4 + 64 * 4)
      return b;
  return 0;
}

// LDS offset (pixel stride kAuxBDs) of (tap, output channel) relative to a window corner.
template <int PW>
__device__ __forceinline__ int auxb_tap_off(int tap, int co) {
  return ((tap >> 2) * PW + (tap & 3)) * kAuxBDs + co;
}

// BYA < AH: work item = (sample, band of BYA A1 rows), staging the 2 BYA + 2 dP rows the band's
// windows read; db2 counts each dP row in one band only (its first 2 BYA rows; the last band
// all of its rows). BYA = AH is the whole-map form.
template <int AH, int AW, int PH, int PW, int BYA = AH>
__global__ __launch_bounds__(kAuxBThreads, 4) void aux_backward2_kernel(float* __restrict__ A1,
                                                                        const float* __restrict__ dP, int n,
                                                                        const float* __restrict__ W2,
                                                                        float* __restrict__ part) {
  constexpr int NBAND = (AH + BYA - 1) / BYA;
  static_assert(PH == 2 * AH + 2 && PW == 2 * AW + 2 && (BYA * AW) % 16 == 0 &&
                    ((AH - (NBAND - 1) * BYA) * AW) % 16 == 0, "k4 s2 transposed conv geometry, whole tiles per band");
  extern __shared__ __attribute__((aligned(16))) float dps[];  // [dP rows of the band][PW][kAuxBDs]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int l16 = lane & 15, lq = lane >> 4;
  // dA1 operands: step u of K (4 + 12 + 12 over the heads), lane k = 4u' + lq. The LDS
  // offsets of heads 1 and 2 repeat every 3 steps one window row down (k = 12j + 4v + lq:
  // tap = 4j + (4v + lq) / 3), so three per lane are kept.
  float wb[28];
#pragma unroll
  for (int u = 0; u < 28; ++u) {
    const int h = u < 4 ? 0 : (u < 16 ? 1 : 2);
    const int k = 4 * (u < 4 ? u : (u < 16 ? u - 4 : u - 16)) + lq;
    const int tap = h == 0 ? k : k / 3;
    const int co = h == 0 ? 0 : (h == 1 ? 1 : 4) + k % 3;
    wb[u] = W2[(16 * h + l16) * 128 + tap * 8 + co];
  }
  int coff[3];
#pragma unroll
  for (int v = 0; v < 3; ++v) coff[v] = auxb_tap_off<PW>((4 * v + lq) / 3, 1 + (4 * v + lq) % 3);
  // dW2 operand B: column l16 of accumulator tile q (head 0: tap; heads 1, 2: 3 taps x co)
  int boff[7];
#pragma unroll
  for (int q = 0; q < 7; ++q) {
    if (q == 0) {
      boff[q] = auxb_tap_off<PW>(l16, 0);
    } else {
      const int col = 16 * ((q - 1) % 3) + l16;
      boff[q] = auxb_tap_off<PW>(col / 3, (q <= 3 ? 1 : 4) + col % 3);
    }
  }
  f4 accw[7];
#pragma unroll
  for (int q = 0; q < 7; ++q) accw[q] = f4zero();
  float db1[3] = {0.0f, 0.0f, 0.0f};
  f4 db2 = f4zero();
  for (int it = blockIdx.x; it < n * NBAND; it += gridDim.x) {
    const int s = it / NBAND, y0 = (it - (it / NBAND) * NBAND) * BYA;
    const int rows = min(BYA, AH - y0);                 // A1 rows of the band
    const int NPX = rows * AW, NT = NPX / 16;           // its pixels, tiles
    const int NPP = (2 * rows + 2) * PW;                // dP pixels staged (rows 2 y0 ..)
    const int NPPC = (y0 + rows == AH ? 2 * rows + 2 : 2 * rows) * PW;  // the ones db2 counts
    const f4* src = reinterpret_cast<const f4*>(dP + ((int64_t)s * PH + 2 * y0) * PW * kAuxC2);
    for (int i = tid; i < NPP * 2; i += kAuxBThreads) {
      const f4 v = src[i];
      float* d = dps + (i >> 1) * kAuxBDs + (i & 1) * 4;
      d[0] = v[0];
      d[1] = v[1];
      d[2] = v[2];
      d[3] = v[3];
      if ((i >> 1) < NPPC) db2 += v;
    }
    __syncthreads();
    float* a1 = A1 + ((int64_t)s * AH + y0) * AW * kAuxC1;
    for (int t = wave; t < NT; t += kAuxBThreads / 64) {
#pragma unroll 2
      for (int ks = 0; ks < 4; ++ks) {  // dW2 over the tile's pixels, 4 per MFMA
        const int px = 16 * t + 4 * ks + lq;
        const int base = (2 * (px / AW) * PW + 2 * (px % AW)) * kAuxBDs;
        const float* ap = a1 + px * kAuxC1 + l16;
        const float x0 = ap[0], x1 = ap[16], x2 = ap[32];
        float b[7];
#pragma unroll
        for (int q = 0; q < 7; ++q) b[q] = dps[base + boff[q]];
        accw[0] = __builtin_amdgcn_mfma_f32_16x16x4f32(x0, b[0], accw[0], 0, 0, 0);
#pragma unroll
        for (int q = 1; q < 4; ++q) accw[q] = __builtin_amdgcn_mfma_f32_16x16x4f32(x1, b[q], accw[q], 0, 0, 0);
#pragma unroll
        for (int q = 4; q < 7; ++q) accw[q] = __builtin_amdgcn_mfma_f32_16x16x4f32(x2, b[q], accw[q], 0, 0, 0);
      }
      // dA1 of the tile: rows = pixels 16t + l16 (operand A), C rows 16t + 4 lq + r
      const int pa = 16 * t + l16;
      const int abase = (2 * (pa / AW) * PW + 2 * (pa % AW)) * kAuxBDs;
      f4 acc[3] = {f4zero(), f4zero(), f4zero()};
#pragma unroll
      for (int u = 0; u < 4; ++u)  // head 0: tap = 4u + lq (ky = u, kx = lq), channel 0
        acc[0] = __builtin_amdgcn_mfma_f32_16x16x4f32(dps[abase + (u * PW + lq) * kAuxBDs], wb[u], acc[0], 0, 0, 0);
#pragma unroll
      for (int u = 4; u < 28; ++u) {
        const int h = u < 16 ? 1 : 2, up = u - (h == 1 ? 4 : 16);
        const float a = dps[abase + coff[up % 3] + (up / 3) * PW * kAuxBDs + (h == 2 ? 3 : 0)];
        acc[h] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, wb[u], acc[h], 0, 0, 0);
      }
      float* op = a1 + (16 * t + 4 * lq) * kAuxC1 + l16;
      float m[3][4];
#pragma unroll
      for (int h = 0; h < 3; ++h)
#pragma unroll
        for (int r = 0; r < 4; ++r) m[h][r] = op[r * kAuxC1 + 16 * h];
#pragma unroll
      for (int h = 0; h < 3; ++h)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float v = m[h][r] > 0.0f ? acc[h][r] : 0.0f;
          db1[h] += v;
          op[r * kAuxC1 + 16 * h] = v;
        }
    }
    __syncthreads();
  }
  // workgroup reduction in a fixed order: wave by wave into LDS (the staging area is free)
  float* red = dps;  // [7][4][64] dW2, [48] db1, [8] db2
#pragma unroll
  for (int h = 0; h < 3; ++h) {
    db1[h] += __shfl_xor(db1[h], 16);
    db1[h] += __shfl_xor(db1[h], 32);
  }
#pragma unroll
  for (int o = 2; o < 64; o <<= 1)
#pragma unroll
    for (int c = 0; c < 4; ++c) db2[c] += __shfl_xor(db2[c], o);
  for (int w = 0; w < kAuxBThreads / 64; ++w) {
    if (wave == w) {
#pragma unroll
      for (int q = 0; q < 7; ++q)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float* d = red + (q * 4 + r) * 64 + lane;
          *d = (w == 0 ? 0.0f : *d) + accw[q][r];
        }
      if (lane < 16) {
#pragma unroll
        for (int h = 0; h < 3; ++h) {
          float* d = red + 7 * 4 * 64 + 16 * h + lane;
          *d = (w == 0 ? 0.0f : *d) + db1[h];
        }
      }
      if (lane < 2) {
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          float* d = red + 7 * 4 * 64 + kAuxC1 + 4 * lane + c;
          *d = (w == 0 ? 0.0f : *d) + db2[c];
        }
      }
    }
    __syncthreads();
  }
  for (int i = tid; i < kAuxBPart; i += kAuxBThreads) part[(int64_t)blockIdx.x * kAuxBPart + i] = red[i];
}

// dW2 [48][16][8] (zeros off the head blocks), db1 [48], db2 [8] from the partials: one
// wave per output, lane-strided over the workgroups and a fixed shuffle tree.
__global__ void aux_backward2_finish_kernel(const float* __restrict__ part, int nblk, float* __restrict__ dW2,
                                            float* __restrict__ db1, float* __restrict__ db2) {
  const int idx = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64, lane = threadIdx.x & 63;
  constexpr int NW = kAuxC1 * 16 * kAuxC2;
  if (idx >= NW + kAuxC1 + kAuxC2) return;
  int src;
  if (idx < NW) {
    const int ci = idx / 128, tap = (idx / 8) % 16, co = idx % 8, h = ci / 16;
    if (aux_head_of_out(co) != h) {
      if (lane == 0) dW2[idx] = 0.0f;
      return;
    }
    int q, col;
    if (h == 0) {
      q = 0;
      col = tap;
    } else {
      const int c3 = tap * 3 + co - (h == 1 ? 1 : 4);
      q = 1 + 3 * (h - 1) + c3 / 16;
      col = c3 % 16;
    }
    const int cl = ci % 16;
    src = (q * 4 + (cl & 3)) * 64 + 16 * (cl >> 2) + col;
  } else {
    src = 7 * 4 * 64 + (idx - NW);
  }
  float s = 0.0f;
  for (int b = lane; b < nblk; b += 64) s += part[(int64_t)b * kAuxBPart + src];
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  if (lane != 0) return;
  if (idx < NW)
    dW2[idx] = s;
  else if (idx < NW + kAuxC1)
    db1[idx - NW] = s;
  else
    db2[idx - NW - kAuxC1] = s;
}

}  // namespace vn
