// vn_conv1.h — conv1 (Conv2d(3->32, k7, s4) on uint8 frames) forward and weight
// gradient, specialised for gfx950 (included by vn_policy.hip after FrameSrc).
//
// The frame(s) of a workgroup are staged once into LDS with 16-B (or 4-B) loads from
// the scene-cache arena rows; operands are then read byte-wise from LDS and converted
// with v_cvt_f32_ubyte (exact integers). Because the conv is linear in x = u/255, the
// 1/255 is applied once to each accumulated sum (epilogue / reduce) instead of to every
// operand — the same fp32 result up to rounding order (parity tests at 1e-5 rel).
// MFMA: v_mfma_f32_32x32x2_f32 (64-cycle issue = 64-cycle dependent latency, so one
// accumulator chain per wave runs at the full rate).
//   forward: D[pixel 32][co 32] += A[pixel][k] * B[k][co]; the 74 B fragments (all of K)
//            stay in registers for the whole kernel; one LDS byte per lane per MFMA.
//   wgrad:   D[co 32][k 32] += A[co][pixel] * B[pixel][k] over 5 k-tiles (148 + bias
//            column); A is read straight from dZ (NHWC: 256 contiguous bytes per wave
//            and step), B from the LDS frame; per-wave partial sums go to slabs that a
//            deterministic reduce sums (and scales by 1/255).
#pragma once

#include <utility>

#include "vn_conv1_lanes.h"

namespace vn {

typedef float f16v __attribute__((ext_vector_type(16)));

template <int W>
__host__ __device__ constexpr int conv1_koff(int k) {
  return k >= 147 ? 0 : (k / 21) * W * 3 + ((k / 3) % 7) * 3 + (k % 3);
}

// f(std::integral_constant<int, 0>{}) ... f(std::integral_constant<int, N - 1>{}): a loop
// whose index is a compile-time constant in every copy of the body
template <class F, int... I>
__device__ __forceinline__ void static_for_impl(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, class F>
__device__ __forceinline__ void static_for(F&& f) {
  static_for_impl(f, std::make_integer_sequence<int, N>{});
}

// Frame f of a wave-uniform work item (every caller's f is uniform). The arena row index is
// read with a scalar load (constant address space: lgkmcnt): as a vector load its address
// dependence made the wave wait for vmcnt(0) — for every load and store in flight, e.g. the
// weight gradient's dZ prefetch — at each call.
__device__ __forceinline__ const uint8_t* frame_ptr(const FrameSrc& src, int f) {
  f = __builtin_amdgcn_readfirstlane(f);
  const int smp = f >> 1, h = f & 1;
  typedef __attribute__((address_space(4))) const int32_t cint32;
  // branch-free (a branch between a load and its use costs the compiler its wait counts):
  // without a rows table the load reads the frame base instead, and its value is not used
  const int32_t* rp = src.rows[h];
  const int32_t* a = rp ? rp + smp : reinterpret_cast<const int32_t*>(src.base[h]);
  const int32_t v = *(cint32*)a;
  const int64_t row = rp ? (int64_t)v : (int64_t)smp;
  return src.base[h] + row * src.stride;
}

// Copy FB bytes of one frame into LDS with NT threads.
template <int FB, int NT>
__device__ __forceinline__ void stage_frame(uint8_t* dst, const uint8_t* src, int tid) {
  if constexpr (FB % 16 == 0) {
    const uint4* s = reinterpret_cast<const uint4*>(src);
    uint4* d = reinterpret_cast<uint4*>(dst);
#pragma unroll 4
    for (int i = tid; i < FB / 16; i += NT) d[i] = s[i];
  } else {
    static_assert(FB % 4 == 0, "frame bytes must be a multiple of 4");
    const uint32_t* s = reinterpret_cast<const uint32_t*>(src);
    uint32_t* d = reinterpret_cast<uint32_t*>(dst);
#pragma unroll 4
    for (int i = tid; i < FB / 4; i += NT) d[i] = s[i];
  }
}

__device__ __forceinline__ float u8f(const uint8_t* p) { return (float)(*p); }

// ---- forward ------------------------------------------------------------------
// NF frames per workgroup iteration, 5 waves; rows = pixels of the NF frames.
template <int H, int W, int OH, int OW, int NF>
__global__ __launch_bounds__(320) void conv1_fwd_kernel(FrameSrc src, int n_frames, const float* __restrict__ Wt,
                                                        const float* __restrict__ bias, float* __restrict__ Y,
                                                        uint32_t* __restrict__ mask) {
  constexpr int FB = H * W * 3;
  constexpr int FBP = (FB + 15) / 16 * 16;
  constexpr int NPIX = OH * OW;
  constexpr int TILES = (NF * NPIX + 31) / 32;
  constexpr int NW = 5;
  __shared__ __attribute__((aligned(16))) uint8_t fr[NF * FBP];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int h = lane >> 5, c32 = lane & 31;
  float b[74];
#pragma unroll
  for (int s = 0; s < 74; ++s) b[s] = (2 * s + h < 147) ? Wt[c32 * 148 + 2 * s + h] : 0.0f;  // k = 147 is padding
  const float bs = bias[c32];
  for (int f0 = blockIdx.x * NF; f0 < n_frames; f0 += gridDim.x * NF) {
    const int nf = min(NF, n_frames - f0);
    for (int j = 0; j < nf; ++j) stage_frame<FB, 320>(fr + j * FBP, frame_ptr(src, f0 + j), tid);
    __syncthreads();
    for (int t = wave; t < TILES; t += NW) {
      const int row = t * 32 + c32;
      const int sel = row / NPIX, px = row - (row / NPIX) * NPIX;
      const int oy = px / OW, ox = px - (px / OW) * OW;
      const uint8_t* base = fr + (sel < nf ? sel : 0) * FBP + (oy * 4 * W + ox * 4) * 3;
      f16v acc;
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[r] = 0.0f;
#pragma unroll
      for (int s = 0; s < 74; ++s) {
        const int k0 = conv1_koff<W>(2 * s), k1 = conv1_koff<W>(2 * s + 1);
        const float a = u8f(base + (h ? k1 : k0));
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b[s], acc, 0, 0, 0);
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int rr = t * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        const float y = fmaxf(acc[r] * (1.0f / 255.0f) + bs, 0.0f);
        // ReLU bitmask: lanes 0-31 (h = 0) and 32-63 (h = 1) are the 32 channels of two pixels
        const uint64_t bal = __ballot(y > 0.0f);
        if (rr < nf * NPIX) {
          Y[((int64_t)f0 * NPIX + rr) * 32 + c32] = y;
          if (c32 == 0) mask[(int64_t)f0 * NPIX + rr] = (uint32_t)(bal >> (32 * h));
        }
      }
    }
    __syncthreads();
  }
}

// ---- forward on bf16 MFMA with split weights ------------------------------------
// The frame bytes are integers 0..255, exact in bf16; each fp32 weight is split by
// truncation into three bf16 terms with w == hi + mid + lo exactly, so every product is
// exact in fp32 and v_mfma_f32_32x32x16_bf16 (16x the f32 MFMA rate) accumulates the same
// sum of exact products as the f32 path, in a different order (parity at 1e-5 rel, as the
// f32 kernel). Three accumulators (one per term) keep three independent MFMA chains.
// K is relaid k' = ky*24 + kr (kr = kx*3 + c < 21, 21..23 and ky = 7 zero-weighted) so
// the 8 k' of a lane's fragment are 8 consecutive frame bytes of one image row: the
// frame is staged into LDS as bf16 rows of RS elements and a fragment is two aligned
// 8-byte LDS reads; the split weights sit in LDS as per-lane fragments (one ds_read_b128
// each), and the next work item's bytes are prefetched into registers.
// Work item = (frame, band of BR output rows): a band stages the 4*BR + 4 image rows its
// taps read (row 4*BR + 3 is the zero-weighted ky = 7 of the band's last row). BR is the
// whole map when the bf16 frame fits next to the weights in half the LDS (84x84: one
// band, two workgroups per CU), else the map is cut into equal bands that do (174x174:
// 9,9,9,9,6 rows). Frame rows of an odd byte count take the f32 kernel.
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

constexpr int kConv1X3WeightLds = 11 * 3 * 64 * 16;  // split weight fragments [slice][term][lane]

template <int H, int W>
struct Conv1X3Band {
  static constexpr int RB = W * 3, RS = (RB + 3) / 4 * 4;  // row bytes; LDS row stride (bf16)
  static constexpr int OH = (H - 7) / 4 + 1;
  static constexpr int rows_of(int br) { return 4 * br + 4 < H ? 4 * br + 4 : H; }
  static constexpr size_t lds_of(int br) { return (size_t)rows_of(br) * RS * 2 + kConv1X3WeightLds; }
  static constexpr int br_max() {
    int br = OH;
    while (br > 1 && lds_of(br) > 80 * 1024) --br;
    return br;
  }
  static constexpr int NB = (OH + br_max() - 1) / br_max();  // bands per frame
  static constexpr int BR = (OH + NB - 1) / NB;               // output rows per band
  static constexpr int BRI = rows_of(BR);                     // image rows staged per band
};

template <int H, int W>
constexpr bool conv1_x3_fits() {
  return (W * 3) % 2 == 0 && (size_t)H * W * 3 % 4 == 0 && Conv1X3Band<H, W>::lds_of(Conv1X3Band<H, W>::BR) <= 80 * 1024;
}

__device__ __forceinline__ void split3_bf16(float w, uint16_t& hi, uint16_t& mid, uint16_t& lo) {
  const uint32_t hb = __float_as_uint(w) & 0xffff0000u;
  const float r1 = w - __uint_as_float(hb);  // exact: the low 16 mantissa bits of w
  const uint32_t mb = __float_as_uint(r1) & 0xffff0000u;
  const float r2 = r1 - __uint_as_float(mb);  // exact, <= 8 significant bits
  hi = (uint16_t)(hb >> 16);
  mid = (uint16_t)(mb >> 16);
  lo = (uint16_t)(__float_as_uint(r2) >> 16);
}

// Four frame bytes -> four bf16 (exact integers): v_cvt_f32_ubyte0..3 and one v_perm_b32 per pair
// taking the two upper halves (6 VALU; the shift + and-or form took 8)
__device__ __forceinline__ uint2 u8x4_bf16(uint32_t v) {
  const uint32_t f0 = __float_as_uint((float)(v & 0xffu)), f1 = __float_as_uint((float)((v >> 8) & 0xffu));
  const uint32_t f2 = __float_as_uint((float)((v >> 16) & 0xffu)), f3 = __float_as_uint((float)(v >> 24));
  return uint2{__builtin_amdgcn_perm(f1, f0, 0x07060302u), __builtin_amdgcn_perm(f3, f2, 0x07060302u)};
}

// Dword i of a band of frame rows (RB bytes each, contiguous) into bf16 LDS rows of RS elements:
// byte pairs never straddle a row (RB even); the second pair of the dword that ends a row
// (col + 2 == RB) starts the next one
template <int RB, int RS>
__device__ __forceinline__ void stage_u8x4_bf16(uint16_t* img, int i, uint32_t v) {
  static_assert(RB % 2 == 0, "byte pairs within rows");
  const uint2 p = u8x4_bf16(v);
  const int e = i * 4, row = e / RB, col = e - row * RB;
  uint16_t* d0 = img + row * RS + col;
  if constexpr (RB % 4 == 0) {  // a dword never straddles a row
    *reinterpret_cast<uint2*>(d0) = p;
  } else {
    *reinterpret_cast<uint32_t*>(d0) = p.x;
    *reinterpret_cast<uint32_t*>(d0 + 2 + (col + 2 == RB ? RS - RB : 0)) = p.y;
  }
}

template <int H, int W, int OH, int OW>
__global__ __launch_bounds__(256, 2) void conv1_fwd_x3_kernel(FrameSrc src, int n_frames, FrameList fl,
                                                           const float* __restrict__ Wt,
                                                           const float* __restrict__ bias, float* __restrict__ Y,
                                                           uint32_t* __restrict__ mask) {
  using B = Conv1X3Band<H, W>;
  constexpr int RB = B::RB, RS = B::RS, BR = B::BR, NB = B::NB, BRI = B::BRI;
  constexpr int NPIX = OH * OW;
  constexpr int TILES = (BR * OW + 31) / 32;  // tiles of a full band
  constexpr int NS = 11;                      // k' slices of 16 (k' < 176)
  constexpr int ND = BRI * RB / 4;            // dwords of a full band
  constexpr int NPF = (ND + 255) / 256;       // prefetched dwords per thread
  static_assert(RB % 2 == 0 && (BRI * RB) % 4 == 0, "band rows of whole dwords");
  // LDS: the band's bf16 image rows, then the split weights as per-lane 16-B fragments [s][term][lane]
  __shared__ __attribute__((aligned(16))) uint16_t img[BRI * RS];
  __shared__ __attribute__((aligned(16))) bf16x8 bw[NS * 3 * 64];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int h = lane >> 5, c32 = lane & 31;
  for (int i = tid; i < NS * 64; i += 256) {  // fragment of slice sl for lane ln
    const int sl = i >> 6, ln = i & 63, hh = ln >> 5, co = ln & 31;
    union { uint16_t u[8]; bf16x8 v; } t0, t1, t2;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int kp = 16 * sl + 8 * hh + j, ky = kp / 24, kr = kp % 24;
      const float w = (ky < 7 && kr < 21) ? Wt[co * 148 + ky * 21 + kr] : 0.0f;
      split3_bf16(w, t0.u[j], t1.u[j], t2.u[j]);
    }
    bw[(sl * 3 + 0) * 64 + ln] = t0.v;
    bw[(sl * 3 + 1) * 64 + ln] = t1.v;
    bw[(sl * 3 + 2) * 64 + ln] = t2.v;
  }
  f4 bs[4];  // the transposed tile's lane holds channels 8j + 4h .. +3 (j = 0..3) of pixel c32
#pragma unroll
  for (int j = 0; j < 4; ++j) bs[j] = *reinterpret_cast<const f4*>(bias + 8 * j + 4 * h);
  // land the bias now: its first use sits in the tile loop's epilogue, where the compiler
  // cannot tell it from the next item's prefetch in flight and waits for vmcnt(0) each tile
#pragma unroll
  for (int j = 0; j < 4; ++j) asm volatile("" ::"v"(bs[j][0]), "v"(bs[j][1]), "v"(bs[j][2]), "v"(bs[j][3]));
  const int n_items = fl_count(fl, n_frames) * NB;
  // dwords of item it's band: rows 4*BR*band .. (clamped to the frame)
  auto band_dwords = [&](int band) { return min(BRI, H - 4 * BR * band) * RB / 4; };
  uint32_t pre[NPF];  // next item's bytes, in flight while the current item computes
  auto load_item = [&](int it) {
    const int f = fl_frame(fl, it / NB), band = it - (it / NB) * NB;
    const uint32_t* s4 = reinterpret_cast<const uint32_t*>(frame_ptr(src, f) + (int64_t)4 * BR * band * RB);
    const int nd = band_dwords(band);
    // unconditional (a lane past the band reloads its last dword; past the last item the item
    // repeats): no branch around the loads for the wait counts to get lost in
#pragma unroll
    for (int j = 0; j < NPF; ++j) pre[j] = s4[min(tid + j * 256, nd - 1)];
  };
  if ((int)blockIdx.x < n_items) load_item(blockIdx.x);
  for (int it = blockIdx.x; it < n_items; it += gridDim.x) {
    const int f = fl_frame(fl, it / NB), band = it - (it / NB) * NB;
    const int oy0 = BR * band, nr = min(BR, OH - oy0), npb = nr * OW;
    const int nd = band_dwords(band);
#pragma unroll
    for (int j = 0; j < NPF; ++j) {  // u8 -> bf16 rows
      const int i = tid + j * 256;
      if (i < nd) stage_u8x4_bf16<RB, RS>(img, i, pre[j]);
    }
    __syncthreads();
    load_item(min(it + (int)gridDim.x, n_items - 1));
    const int tiles = (npb + 31) / 32;
    for (int t = wave; t < tiles; t += 4) {
      const int px = min(t * 32 + c32, npb - 1);
      const int oy = px / OW, ox = px - (px / OW) * OW;
      const uint16_t* base = img + (oy * 4) * RS + ox * 12;
      // opaque per tile: keeps the 33 weight-fragment reads inside the tile loop (hoisted,
      // they would hold 132 VGPRs across it and spill)
      int wl = lane;
      asm volatile("" : "+v"(wl));
      f16v acc[3];
#pragma unroll
      for (int p = 0; p < 3; ++p)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[p][r] = 0.0f;
#pragma unroll
      for (int sl = 0; sl < NS; ++sl) {
        const int k0 = 16 * sl + 8 * h, ky = k0 / 24, kr0 = k0 - (k0 / 24) * 24;
        const uint2* q = reinterpret_cast<const uint2*>(base + ky * RS + kr0);
        union { uint2 u[2]; bf16x8 v; } a;
        a.u[0] = q[0];
        a.u[1] = q[1];
#pragma unroll
        for (int p = 0; p < 3; ++p)  // D^T = W^T A^T: rows = channels, columns = pixels
          acc[p] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bw[(sl * 3 + p) * 64 + wl], a.v, acc[p], 0, 0, 0);
      }
      // lane (pixel c32, h) holds channels 8j + 4h + (0..3): four 16-B stores per lane; the
      // ReLU bits of the other 16 channels come from the partner lane (c32, 1 - h)
      const int rr = t * 32 + c32;
      const int64_t pix = (int64_t)f * NPIX + oy0 * OW + rr;
      uint32_t bits = 0;
      f4 y[4];
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int i = 4 * j + r;
          const float sum = (acc[2][i] + acc[1][i]) + acc[0][i];
          y[j][r] = fmaxf(sum * (1.0f / 255.0f) + bs[j][r], 0.0f);
          bits |= (y[j][r] > 0.0f ? 1u : 0u) << (8 * j + 4 * h + r);
        }
      bits |= (uint32_t)__shfl_xor((int)bits, 32);
      if (rr < npb) {
#pragma unroll
        for (int j = 0; j < 4; ++j) *reinterpret_cast<f4*>(Y + pix * 32 + 8 * j + 4 * h) = y[j];
        if (h == 0) mask[pix] = bits;
      }
    }
    __syncthreads();
  }
  (void)TILES;
}

// conv1_fwd_x3_kernel with the split weights resident in registers (round 6). The per-tile
// budget of the LDS-fragment form (tools/isa_budget.py, 174x174): 33 MFMAs, 44 LDS reads (33 of
// them the weight fragments, each waited on right before its MFMA: lgkmcnt(0/1) x 33), ~150
// VALU; per item 21 prefetch loads at ~6.5 address instructions each and a branch per staged
// dword. Here a lane's 33 fragments (132 VGPRs) are split once per kernel, so a tile reads only
// its 11 image fragments; the next item's band is prefetched through a buffer descriptor over
// the band (dwords past it read as zero: one address per thread, no clamps); the ReLU bits
// are med3(bits(y), 0, 1) << (8j + r), shifted once by 4h. Same products, same three chains and
// the same final sum as conv1_fwd_x3_kernel: bitwise equal outputs.
template <int H, int W, int OH, int OW>
__global__ __launch_bounds__(256, 2) void conv1_fwd_x3r_kernel(FrameSrc src, int n_frames, FrameList fl,
                                                            const float* __restrict__ Wt,
                                                            const float* __restrict__ bias, float* __restrict__ Y,
                                                            uint32_t* __restrict__ mask) {
  using B = Conv1X3Band<H, W>;
  // the band's bf16 rows back to back (row stride RB elements, not B::RS): staged dword i is
  // image elements 4i .. 4i + 3, one 8-byte store at 8i with no row arithmetic; at 174x174
  // (522 B rows) a fragment is then only 4-byte aligned and is read as four dwords
  constexpr int RB = B::RB, RS = RB, BR = B::BR, NB = B::NB, BRI = B::BRI;
  constexpr int NPIX = OH * OW;
  constexpr int NS = 11;                // k' slices of 16 (k' < 176)
  constexpr int ND = BRI * RB / 4;      // dwords of a full band
  constexpr int NPF = (ND + 255) / 256;  // prefetched dwords per thread
  static_assert(RB % 2 == 0 && (BRI * RB) % 4 == 0, "band rows of whole dwords");
  __shared__ __attribute__((aligned(16))) uint16_t img[BRI * RS];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int h = lane >> 5, c32 = lane & 31;
  bf16x8 bw[NS][3];  // lane (h, co = c32): k' = 16 sl + 8h + j of output channel co
#pragma unroll
  for (int sl = 0; sl < NS; ++sl) {
    union { uint16_t u[8]; bf16x8 v; } t0, t1, t2;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int kp = 16 * sl + 8 * h + j, ky = kp / 24, kr = kp - (kp / 24) * 24;
      const float w = (ky < 7 && kr < 21) ? Wt[c32 * 148 + ky * 21 + kr] : 0.0f;
      split3_bf16(w, t0.u[j], t1.u[j], t2.u[j]);
    }
    bw[sl][0] = t0.v;
    bw[sl][1] = t1.v;
    bw[sl][2] = t2.v;
  }
  f4 bs[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) bs[j] = *reinterpret_cast<const f4*>(bias + 8 * j + 4 * h);
#pragma unroll
  for (int j = 0; j < 4; ++j) asm volatile("" ::"v"(bs[j][0]), "v"(bs[j][1]), "v"(bs[j][2]), "v"(bs[j][3]));
  const int n_items = fl_count(fl, n_frames) * NB;
  auto band_dwords = [&](int band) { return min(BRI, H - 4 * BR * band) * RB / 4; };
  uint32_t pre[NPF];
  auto load_item = [&](int it) {
    const int f = fl_frame(fl, it / NB), band = it - (it / NB) * NB;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(frame_ptr(src, f) + (int64_t)4 * BR * band * RB), 0, band_dwords(band) * 4, 0x00020000);
#pragma unroll
    for (int j = 0; j < NPF; ++j) {
      pre[j] = __builtin_amdgcn_raw_buffer_load_b32(rs, 4 * tid + 1024 * j, 0, 0);
      // issue order = use order, so the staging below waits vmcnt(NPF - 1 - j) for dword j (the
      // scheduler's own order made it one vmcnt(0): every tile store of the item in flight too)
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  auto stage = [&]() {
#pragma unroll
    for (int j = 0; j < NPF; ++j) {  // u8 -> bf16 rows (dwords past a short band are zeros)
      const int i = tid + j * 256;
      if (j + 1 < NPF || i < ND) *reinterpret_cast<uint2*>(img + 4 * i) = u8x4_bf16(pre[j]);
    }
  };
  if ((int)blockIdx.x < n_items) load_item(blockIdx.x);
  for (int it = blockIdx.x; it < n_items; it += gridDim.x) {
    const int f = fl_frame(fl, it / NB), band = it - (it / NB) * NB;
    const int oy0 = BR * band, nr = min(BR, OH - oy0), npb = nr * OW;
    stage();
    __syncthreads();
    load_item(min(it + (int)gridDim.x, n_items - 1));
    const int tiles = (npb + 31) / 32;
    auto tile = [&](int t) {
      const int px = min(t * 32 + c32, npb - 1);
      const int oy = px / OW, ox = px - (px / OW) * OW;
      const uint16_t* base = img + (oy * 4) * RS + ox * 12;
      f16v acc[3];
#pragma unroll
      for (int p = 0; p < 3; ++p)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[p][r] = 0.0f;
#pragma unroll
      for (int sl = 0; sl < NS; ++sl) {
        const int k0 = 16 * sl + 8 * h, ky = k0 / 24, kr0 = k0 - (k0 / 24) * 24;
        union { uint2 u[2]; uint32_t d[4]; bf16x8 v; } a;
        if constexpr (RS % 4 == 0) {
          const uint2* q = reinterpret_cast<const uint2*>(base + ky * RS + kr0);
          a.u[0] = q[0];
          a.u[1] = q[1];
        } else {
          const uint32_t* q = reinterpret_cast<const uint32_t*>(base + ky * RS + kr0);
#pragma unroll
          for (int e = 0; e < 4; ++e) a.d[e] = q[e];
        }
#pragma unroll
        for (int p = 0; p < 3; ++p) acc[p] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bw[sl][p], a.v, acc[p], 0, 0, 0);
      }
      const int rr = t * 32 + c32;
      const int64_t pix = (int64_t)f * NPIX + oy0 * OW + rr;
      uint32_t bits = 0;
      f4 y[4];
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int i = 4 * j + r;
          const float sum = (acc[2][i] + acc[1][i]) + acc[0][i];
          y[j][r] = fmaxf(sum * (1.0f / 255.0f) + bs[j][r], 0.0f);
          // med3(bits(y), 0, 1) as int: 1 <=> y > 0 (y = fmaxf(., 0) is never NaN; -0 reads as 0);
          // as C the compiler makes it v_cmp + v_cndmask of a constant + s_nop for the VCC hazard
          uint32_t one;
          asm("v_med3_i32 %0, %1, 0, 1" : "=v"(one) : "v"(y[j][r]));
          bits |= one << (8 * j + r);
        }
      bits <<= 4 * h;
      bits |= (uint32_t)__shfl_xor((int)bits, 32);
      if (rr < npb) {
#pragma unroll
        for (int j = 0; j < 4; ++j) *reinterpret_cast<f4*>(Y + pix * 32 + 8 * j + 4 * h) = y[j];
        if (h == 0) mask[pix] = bits;
      }
    };
    for (int t = wave; t < tiles; t += 4) tile(t);
    __syncthreads();
  }
}

// ---- weight gradient ----------------------------------------------------------
// One frame per workgroup iteration, its pixels in chunks of CP: the chunk's dZ rows
// (CP x 32 fp32, 16-B loads) and the frame bytes are staged into LDS together, then each
// of the 4 waves reduces over a quarter of the chunk, two pixels per MFMA step.
// Columns: k in [0,147) data, 147 pad, 148 = bias (ones), 149..159 zero.
template <int H, int W, int OH, int OW, int CP>
__global__ __launch_bounds__(256) void conv1_wgrad_kernel(FrameSrc src, int n_frames, const float* __restrict__ dZ,
                                                          float* __restrict__ slab) {
  constexpr int FB = H * W * 3;
  constexpr int FBP = (FB + 15) / 16 * 16;
  constexpr int NPIX = OH * OW;
  static_assert(CP % 8 == 0, "chunk must split into 4 waves x 2 pixels");
  constexpr int SPW = CP / 8;  // MFMA steps per wave per chunk
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  uint8_t* fr = smem;
  float* dzs = reinterpret_cast<float*>(smem + FBP);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int h = lane >> 5, c32 = lane & 31;
  int koff[5];
#pragma unroll
  for (int nt = 0; nt < 5; ++nt) koff[nt] = conv1_koff<W>(nt * 32 + c32);
  const int k4 = 128 + c32;
  const float mul4 = k4 < 147 ? 1.0f : 0.0f;
  const float add4 = k4 == 148 ? 1.0f : 0.0f;
  f16v acc[5];
#pragma unroll
  for (int nt = 0; nt < 5; ++nt)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[nt][r] = 0.0f;
  for (int f = blockIdx.x; f < n_frames; f += gridDim.x) {
    const float* dzf = dZ + (int64_t)f * NPIX * 32;
    for (int c0 = 0; c0 < NPIX; c0 += CP) {
      const int np = min(CP, NPIX - c0);
      {
        const f4* s4 = reinterpret_cast<const f4*>(dzf + (int64_t)c0 * 32);
        f4* d4 = reinterpret_cast<f4*>(dzs);
        for (int i = tid; i < np * 8; i += 256) d4[i] = s4[i];
      }
      if (c0 == 0) stage_frame<FB, 256>(fr, frame_ptr(src, f), tid);
      __syncthreads();
#pragma unroll 5
      for (int s = 0; s < SPW; ++s) {
        const int pl = wave * (CP / 4) + 2 * s + h;
        const bool valid = pl < np;
        const float a = valid ? dzs[pl * 32 + c32] : 0.0f;
        const int p = valid ? c0 + pl : 0;
        const int oy = p / OW, ox = p - (p / OW) * OW;
        const uint8_t* pb = fr + (oy * 4 * W + ox * 4) * 3;
#pragma unroll
        for (int nt = 0; nt < 4; ++nt)
          acc[nt] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, u8f(pb + koff[nt]), acc[nt], 0, 0, 0);
        const float b4 = fmaf(u8f(pb + koff[4]), mul4, add4);
        acc[4] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b4, acc[4], 0, 0, 0);
      }
      __syncthreads();
    }
  }
  // D[co = row][k = nt*32 + c32]
  float* out = slab + ((int64_t)blockIdx.x * 4 + wave) * (32 * 160);
#pragma unroll
  for (int nt = 0; nt < 5; ++nt)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int co = (r & 3) + 8 * (r >> 2) + 4 * h;
      out[co * 160 + nt * 32 + c32] = acc[nt][r];
    }
}

template <int H, int W, int CP>
constexpr size_t conv1_wgrad_lds() {
  return (size_t)(H * W * 3 + 15) / 16 * 16 + (size_t)CP * 32 * 4;
}

__global__ void conv1_wgrad_reduce_kernel(const float* __restrict__ slab, int nslab, float* dW, float* db) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;  // co*160 + k
  if (idx >= 32 * 160) return;
  const int co = idx / 160, k = idx - (idx / 160) * 160;
  if (k > 148) return;
  float s = 0.0f;
  for (int z = 0; z < nslab; ++z) s += slab[(int64_t)z * 32 * 160 + idx];
  if (k < 148)
    dW[co * 148 + k] = k < 147 ? s * (1.0f / 255.0f) : 0.0f;
  else
    db[co] = s;
}

// ---- weight gradient on bf16 MFMA with split dZ ----------------------------------
// D[co 32][tap 32] += A[co][pixel 16] * B[pixel 16][tap] on v_mfma_f32_32x32x16_bf16, five
// tap tiles (147 taps + bias column): dZ is split by truncation into three bf16 terms
// (exact, as the forward's weights), the frame bytes are exact in bf16, so every product is
// exact and the fp32 accumulation sees the same terms as the f32 kernel.
//   A: read straight from dZ in its MFMA layout — lane (co, h) takes the 8 pixels of group
//      g = 2s + h (one output row's pixels 8(g % GPR) .. +7, the last group of a row
//      padding with dZ = 0): eight loads of one 128-B pixel row each, two steps ahead.
//   B: the frame is staged as Q[y][x & 3][c][x >> 2] (bf16, strides PC / PX / RSQ elements
//      of the layout), so the 8 pixels of a group at one tap (ky, kx, c) are 8 consecutive
//      elements: one ds_read_b128 per tile (taps kx >= 4 sit in tiles 3-4 and take one more
//      element and a 16-bit funnel shift). The tap -> lane tables (vn_conv1_lanes.h, one per
//      layout) put the 16 lanes of every b128 pass group on distinct bank quads.
// Work item = (frame, band of BR output rows); a band stages the 4*BR + 3 image rows its taps
// read (84x84: the whole frame in one band; 174x174: 6 bands of 7 rows; 300x400: 19 of 4).
// Wave w takes the steps s = w (mod 4) of every band; the four wave sums are folded through
// LDS into one slab per workgroup, slot tile*32 + c32 (kConv1WgradCol maps it to dW).
template <int H, int W>
struct Conv1WgQ;  // Q strides (bf16 elements) and the lane-table layout id
template <>
struct Conv1WgQ<84, 84> {
  static constexpr int PC = 24, PX = 72, RSQ = 296, ID = 0;
};
template <>
struct Conv1WgQ<174, 174> {
  static constexpr int PC = 72, PX = 216, RSQ = 888, ID = 1;
};
template <>
struct Conv1WgQ<300, 400> {
  static constexpr int PC = 120, PX = 360, RSQ = 1464, ID = 2;
};

template <int H, int W>
struct Conv1WgBand {
  using Q = Conv1WgQ<H, W>;
  static constexpr int OH = (H - 7) / 4 + 1, OW = (W - 7) / 4 + 1;
  static constexpr int GPR = (OW + 7) / 8;  // 8-pixel groups per output row
  static constexpr int rows_of(int br) { return 4 * br + 3 < H ? 4 * br + 3 : H; }
  static constexpr size_t lds_of(int br) { return (size_t)rows_of(br) * Q::RSQ * 2; }
  static constexpr int br_max() {
    int br = OH;
    while (br > 1 && lds_of(br) > 56 * 1024) --br;
    return br;
  }
  static constexpr int NB = (OH + br_max() - 1) / br_max();
  static constexpr int BR = (OH + NB - 1) / NB;
  static constexpr int BRI = rows_of(BR);
  static constexpr size_t LDS = lds_of(BR) > 32 * 160 * 4 ? lds_of(BR) : 32 * 160 * 4;  // + the final fold
};

template <int H, int W>
constexpr bool conv1_wgrad_x3_fits() {
  return (H == 84 && W == 84) || (H == 174 && W == 174) || (H == 300 && W == 400);
}

// dst = the lanes of mask m ? v : 0 (v_cndmask on an SGPR-pair lane mask: one VALU, no compare)
__device__ __forceinline__ float select_lanes(float v, uint64_t m) {
  float r;
  asm("v_cndmask_b32_e64 %0, 0, %1, %2" : "=v"(r) : "v"(v), "s"(m));
  return r;
}

// LEAN (round 6; tools/isa_budget.py put the 174x174 step at ~103 VALU for 15 MFMAs): the dZ
// validity of a step depends only on the lane's half (g = 2s + h), so it is two scalar pixel
// counts and one v_cndmask per value on an SGPR lane mask (was a compare + cndmask per value);
// the B fragments of pad slots are left as read (finite staged bytes; their accumulator slots
// are never read: kConv1WgradCol -1) and the bias lane reads 8 bf16 ones kept in LDS past the
// fold area instead of masking every tile-2 fragment (12 VALU per step). dW / db bitwise equal.
template <int H, int W, int OH, int OW, bool LEAN = false>
__global__ __launch_bounds__(256) void conv1_wgrad_x3_kernel(FrameSrc src, int n_frames, FrameList fl,
                                                             const float* __restrict__ dZ, float* __restrict__ slab) {
  using Bd = Conv1WgBand<H, W>;
  using QL = typename Bd::Q;
  constexpr int PC = QL::PC, PX = QL::PX, RSQ = QL::RSQ;
  constexpr int RB = W * 3;
  constexpr int NPIX = OH * OW;
  constexpr int GPR = Bd::GPR, BR = Bd::BR, NB = Bd::NB, BRI = Bd::BRI;
  constexpr int PAIRS = (W + 7) / 8;  // 8-pixel (x) staging pairs per image row (the last one partial)
  constexpr int NT = (BRI * PAIRS + 255) / 256;
  constexpr int NDW = RB % 4 == 0 ? 6 : 7;  // dwords per staging task (7: rows start at 2 mod 4)
  static_assert(OH == Bd::OH && OW == Bd::OW, "geometry");
  // staged pairs never overlap; every window read (padding pixels included) stays inside its
  // image row and sees written or zeroed (finite) entries
  static_assert(PX >= 3 * PC && PC >= 2 * PAIRS && 3 * PX + 2 * PC + 8 * GPR < RSQ, "Q strides");
  static_assert(RB % 2 == 0, "even row bytes");
  extern __shared__ __attribute__((aligned(16))) uint8_t smem_wg[];
  uint16_t* Q = reinterpret_cast<uint16_t*>(smem_wg);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int h = lane >> 5, c32 = lane & 31;
  const uint16_t* ones = reinterpret_cast<const uint16_t*>(smem_wg + Bd::LDS);  // LEAN: 8 bf16 ones
  {  // never-written Q entries (x >> 2 >= 2 * PAIRS, row tails) are read by padding pixels: zero
    uint4* q4 = reinterpret_cast<uint4*>(Q);
    for (int i = tid; i < BRI * RSQ / 8; i += 256) q4[i] = uint4{0u, 0u, 0u, 0u};
    if (LEAN && tid == 0) *reinterpret_cast<uint4*>(smem_wg + Bd::LDS) = uint4{0x3f803f80u, 0x3f803f80u, 0x3f803f80u, 0x3f803f80u};
    __syncthreads();  // before any wave stages the first item over the zeroed rows
  }
  int loff[5];
#pragma unroll
  for (int nt = 0; nt < 5; ++nt) {
    const int t = kConv1WgradRead[QL::ID][nt][c32], ky = t / 21, kx = (t / 3) % 7, c = t % 3;
    loff[nt] = ky * RSQ + (kx & 3) * PX + c * PC;
  }
  const int col2 = kConv1WgradCol[QL::ID][2][c32];  // tile 2 carries the bias column and pad lanes
  const uint32_t keep2 = col2 >= 0 && col2 < 147 ? 0xffffffffu : 0u;
  const uint32_t add2 = col2 == 148 ? 0x3f803f80u : 0u;
  const uint32_t keep4 = kConv1WgradCol[QL::ID][4][c32] >= 0 ? 0xffffffffu : 0u;
  const bool bias_lane = col2 == 148;
  const int wv = __builtin_amdgcn_readfirstlane(wave);
  f16v acc[5];
#pragma unroll
  for (int nt = 0; nt < 5; ++nt)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[nt][r] = 0.0f;
  const int n_items = fl_count(fl, n_frames) * NB;
  auto band_rows = [&](int band) { return min(BRI, H - 4 * BR * band); };
  // Every wave runs KW steps of every item (KW a multiple of D: the D dZ register sets rotate across
  // items too), the ones past the band's KS on zeroed dZ; all loads are unconditional, so the
  // compiler counts every wait (a load behind a branch, or a trip count it cannot see, made
  // the waves wait for vmcnt(0): all loads and stores in flight, once per step).
  constexpr int KS_MAX = (BR * GPR + 1) / 2;
  constexpr int KW0 = (KS_MAX + 3) / 4;
  // dZ register sets: step i + D is loaded while steps i + 1 .. i + D - 1 wait; three where KW
  // allows it without an extra masked step (174x174: 6), else two (84x84: 8)
  // LEAN at 174x174 (130 VGPRs + 80 AGPRs): every step of the next item in flight (D = KW = 6)
  constexpr int D = (LEAN && H == 174) ? KW0 : KW0 % 3 == 0 ? 3 : 2;
  constexpr int KW = (KW0 + D - 1) / D * D;
  static_assert(NT <= KW, "staging tasks are issued one per step");
  // staging task (band row y, pair m): pixels 8m .. 8m+7 of the row = 24 frame bytes (fewer
  // in the last pair), prefetched into registers one item ahead as NDW aligned dwords through
  // a buffer descriptor over the frame: the dwords past its end (last pair of the last row)
  // read as zero instead of needing a branch. A task past the band reloads the band's last
  // task (stage_q skips it).
  uint32_t pre[NT][NDW];
  // f: item it's frame (resolved once per item by item_geom)
  auto load_task = [&](int r, int it, int f) {
    const int band = it - (it / NB) * NB;
    const int t = min(tid + r * 256, band_rows(band) * PAIRS - 1);
    const int y = t / PAIRS, m = t - (t / PAIRS) * PAIRS;
    const int off = (4 * BR * band + y) * RB + m * 24;
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc((void*)frame_ptr(src, f), 0, H * W * 3, 0x00020000);
#pragma unroll
    for (int q = 0; q < NDW; ++q) pre[r][q] = __builtin_amdgcn_raw_buffer_load_b32(rs, (off & ~3) + 4 * q, 0, 0);
  };
  auto stage_q = [&](int band) {
#pragma unroll
    for (int r = 0; r < NT; ++r) {
      // a task past the band repeats the band's last task (the same bytes to the same place)
      const int t = min(tid + r * 256, band_rows(band) * PAIRS - 1);
      {
        const int y = t / PAIRS, m = t - (t / PAIRS) * PAIRS;
        uint32_t d[6];
        if constexpr (NDW == 6) {
#pragma unroll
          for (int q = 0; q < 6; ++q) d[q] = pre[r][q];
        } else {
          const int sh = (int)((((int64_t)(4 * BR * band + y) * RB) & 3) * 8);  // 0 or 16
#pragma unroll
          for (int q = 0; q < 6; ++q) d[q] = __builtin_amdgcn_alignbit(pre[r][q + 1], pre[r][q], sh);
        }
        const int nv = min(24, RB - m * 24);  // valid bytes of the pair
#pragma unroll
        for (int q = 0; q < 6; ++q)
          if (4 * q + 4 > nv) d[q] = 4 * q >= nv ? 0u : d[q] & (0xffffffffu >> (8 * (4 * q + 4 - nv)));
        uint32_t* qrow = reinterpret_cast<uint32_t*>(Q + y * RSQ + 2 * m);
#pragma unroll
        for (int rx = 0; rx < 4; ++rx)
#pragma unroll
          for (int c = 0; c < 3; ++c) {
            const int b0 = 3 * rx + c, b1 = b0 + 12;  // pixel rx and rx + 4 of the 8
            const float lo = (float)((d[b0 >> 2] >> (8 * (b0 & 3))) & 0xffu);
            const float hi = (float)((d[b1 >> 2] >> (8 * (b1 & 3))) & 0xffu);
            qrow[(rx * PX + c * PC) / 2] = __builtin_amdgcn_perm(__float_as_uint(hi), __float_as_uint(lo), 0x07060302u);
          }
      }
    }
  };
  // group g's 8 pixels of dZ, unconditionally off one address (a group past the band reloads
  // the band's last group); the step zeroes what is not the group's (z_valid). The last group of
  // a row reads up to 7 pixels past the row: the next row, or past the frame the next sample's
  // map or the activation store's next region (dZ is conv1's slice of it) — in bounds, unused.
  auto load_z = [&](float (&z)[8], int f, int oy0, int ng, int s) {
    const int g = min(2 * s + h, ng - 1), oy = oy0 + g / GPR, ox0 = 8 * (g - (g / GPR) * GPR);
    const float* zf = dZ + ((int64_t)f * NPIX + oy * OW + ox0) * 32 + c32;
#pragma unroll
    for (int j = 0; j < 8; ++j) z[j] = zf[j * 32];
  };
  auto z_valid = [&](int ng, int s) {  // pixels of step s's group that are the band's
    const int g = 2 * s + h, ox0 = 8 * (g - (g / GPR) * GPR);
    return g < ng ? min(8, OW - ox0) : 0;
  };
  auto item_geom = [&](int it, int& f, int& oy0, int& ng) {
    f = fl_frame(fl, it / NB);
    const int band = it - (it / NB) * NB;
    oy0 = BR * band;
    ng = min(BR, OH - oy0) * GPR;
  };
  float zb[D][8];  // dZ of steps i .. i + D - 1 of the wave (step i + D is loaded into i's set)
  if ((int)blockIdx.x < n_items) {
    int f, oy0, ng;
    item_geom(blockIdx.x, f, oy0, ng);
#pragma unroll
    for (int r = 0; r < NT; ++r) load_task(r, blockIdx.x, f);
#pragma unroll
    for (int d = 0; d < D; ++d) load_z(zb[d], f, oy0, ng, wave + 4 * d);
  }
  for (int it = blockIdx.x; it < n_items; it += gridDim.x) {
    int f, oy0, ng;
    item_geom(it, f, oy0, ng);
    const int band = it - (it / NB) * NB;
    stage_q(band);
    __syncthreads();
    const int inext = min(it + (int)gridDim.x, n_items - 1);
    int fn, oy0n, ngn;
    item_geom(inext, fn, oy0n, ngn);
    static_for<KW>([&](auto I) {
      constexpr int i = decltype(I)::value;
      const int s = wave + 4 * i;
      float(&z)[8] = zb[i % D];
      union { uint16_t u[8]; bf16x8 v; } a0, a1, a2;
      if constexpr (LEAN) {
        const int su = wv + 4 * i;  // the wave's step (scalar); half h takes group 2 su + h
        auto nvs = [&](int g) { return g < ng ? min(8, OW - 8 * (g - (g / GPR) * GPR)) : 0; };
        const int nv0 = nvs(2 * su), nv1 = nvs(2 * su + 1);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const uint64_t m = (j < nv0 ? 0xffffffffull : 0ull) | (j < nv1 ? 0xffffffff00000000ull : 0ull);
          split3_bf16(select_lanes(z[j], m), a0.u[j], a1.u[j], a2.u[j]);
        }
      } else {
        const int nvz = z_valid(ng, s);
#pragma unroll
        for (int j = 0; j < 8; ++j) split3_bf16(j < nvz ? z[j] : 0.0f, a0.u[j], a1.u[j], a2.u[j]);
      }
      if constexpr (i < NT) load_task(i, inext, fn);
      if constexpr (i + D < KW)
        load_z(z, f, oy0, ng, s + 4 * D);
      else
        load_z(z, fn, oy0n, ngn, wave + 4 * (i + D - KW));
      const int g = min(2 * s + h, ng - 1);
      const int oy = g / GPR, ox0 = 8 * (g - (g / GPR) * GPR);
      const uint16_t* gb = Q + oy * 4 * RSQ + ox0;
      union { bf16x8 v; uint4 q; uint32_t d[4]; } b[5];
      uint32_t e[2];
#pragma unroll
      for (int nt = 0; nt < 5; ++nt)
        b[nt].q = *reinterpret_cast<const uint4*>(LEAN && nt == 2 && bias_lane ? ones : gb + loff[nt]);
#pragma unroll
      for (int nt = 3; nt < 5; ++nt) e[nt - 3] = gb[loff[nt] + 8];
#pragma unroll
      for (int nt = 3; nt < 5; ++nt) {  // taps kx >= 4 read pixel x >> 2 one further
        const uint32_t d0 = b[nt].d[0], d1 = b[nt].d[1], d2 = b[nt].d[2], d3 = b[nt].d[3];
        b[nt].d[0] = __builtin_amdgcn_alignbit(d1, d0, 16);
        b[nt].d[1] = __builtin_amdgcn_alignbit(d2, d1, 16);
        b[nt].d[2] = __builtin_amdgcn_alignbit(d3, d2, 16);
        b[nt].d[3] = __builtin_amdgcn_alignbit(e[nt - 3], d3, 16);
      }
      if constexpr (!LEAN) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          b[2].d[q] = (b[2].d[q] & keep2) | add2;
          b[4].d[q] &= keep4;
        }
      }
#pragma unroll
      for (int nt = 0; nt < 5; ++nt) acc[nt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0.v, b[nt].v, acc[nt], 0, 0, 0);
#pragma unroll
      for (int nt = 0; nt < 5; ++nt) acc[nt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1.v, b[nt].v, acc[nt], 0, 0, 0);
#pragma unroll
      for (int nt = 0; nt < 5; ++nt) acc[nt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a2.v, b[nt].v, acc[nt], 0, 0, 0);
    });
    __syncthreads();
  }
  // fold the four wave sums in LDS (fixed order), one slab per workgroup: D[co][slot]
  float* red = reinterpret_cast<float*>(Q);
  for (int w = 0; w < 4; ++w) {
    if (wave == w) {
#pragma unroll
      for (int nt = 0; nt < 5; ++nt)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int co = (r & 3) + 8 * (r >> 2) + 4 * h;
          const int ix = co * 160 + nt * 32 + c32;
          red[ix] = w == 0 ? acc[nt][r] : red[ix] + acc[nt][r];
        }
    }
    __syncthreads();
  }
  float* out = slab + (int64_t)blockIdx.x * (32 * 160);
  for (int ix = tid; ix < 32 * 160 / 4; ix += 256)
    reinterpret_cast<f4*>(out)[ix] = reinterpret_cast<const f4*>(red)[ix];
}

// dW / db from the slot-ordered partial sums of conv1_wgrad_x3_kernel (kConv1WgradCol of
// layout `layout`).
__global__ void conv1_wgrad_x3_finish_kernel(const float* __restrict__ part, int nparts, int layout, float* dW,
                                             float* db) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;  // co*160 + slot
  if (idx >= 32 * 160) return;
  const int co = idx / 160, slot = idx - (idx / 160) * 160;
  const int col = kConv1WgradCol[layout][slot >> 5][slot & 31];
  if (col < 0) return;
  float s = 0.0f;
  for (int z = 0; z < nparts; ++z) s += part[(int64_t)z * 32 * 160 + idx];
  if (col < 147)
    dW[co * 148 + col] = s * (1.0f / 255.0f);
  else
    db[co] = s;
  if (col == 148) dW[co * 148 + 147] = 0.0f;  // k = 147 is padding
}

// Deterministic two-stage sum of nslab slabs of n floats: stage 1 sums the slabs z = y
// (mod gridDim.y) per column into partial[y]; stage 2 (conv1_wgrad_finish_kernel or
// sum_slabs_kernel) sums the partials in order.
__global__ void slab_partial_kernel(const float* __restrict__ slab, int nslab, int64_t n, float* __restrict__ partial) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float s = 0.0f;
  for (int z = blockIdx.y; z < nslab; z += gridDim.y) s += slab[(int64_t)z * n + i];
  partial[(int64_t)blockIdx.y * n + i] = s;
}

// ---- conv2 weight gradient ----------------------------------------------------
// dW2[co][(ky*4+kx)*32 + ci] = sum over frames and output pixels p of
// dZ2[f][p][co] * X1[f][(2oy+ky)*IW + 2ox+kx][ci]. Work item = (frame, band of BR output
// rows): the band's X1 rows (2*BR + 2 of them) and dZ2 rows are staged in LDS; wave w owns
// taps 4w..4w+3 (four 32x32 accumulators: co x ci), two output pixels per MFMA step.
// 84x84 (20x20 conv1 map) stages the whole frame in one band; 174x174 (42x42) bands of 5
// rows keep two workgroups per CU. Bias gradient: column sums of dZ2 (wave 0).
template <int IH, int IW, int OH, int OW>
struct Conv2WgBand {
  static constexpr int rows_of(int br) { return 2 * br + 2 < IH ? 2 * br + 2 : IH; }
  static constexpr size_t lds_of(int br) {
    return ((size_t)rows_of(br) * IW * 32 + (size_t)(br * OW + 1) / 2 * 2 * 32) * 4;
  }
  static constexpr int br_max() {
    int br = OH;
    while (br > 1 && lds_of(br) > 80 * 1024) --br;
    return br;
  }
  static constexpr int NB = (OH + br_max() - 1) / br_max();
  static constexpr int BR = (OH + NB - 1) / NB;
  static constexpr size_t LDS = lds_of(BR);
};

template <int IH, int IW, int OH, int OW>
constexpr size_t conv2_wgrad_lds() {
  return Conv2WgBand<IH, IW, OH, OW>::LDS;
}

template <int IH, int IW, int OH, int OW>
__global__ __launch_bounds__(256) void conv2_wgrad_kernel(const float* __restrict__ X1, const float* __restrict__ dZ2,
                                                          int n_frames, float* __restrict__ slab,
                                                          float* __restrict__ bias_slab, FrameList fl) {
  using Bd = Conv2WgBand<IH, IW, OH, OW>;
  constexpr int BR = Bd::BR, NB = Bd::NB;
  constexpr int NX = Bd::rows_of(BR) * IW * 32, NP = OH * OW;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  float* xs = reinterpret_cast<float*>(smem);
  float* ds = xs + NX;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int h = lane >> 5, c32 = lane & 31;
  f16v acc[4];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[j][r] = 0.0f;
  float bacc = 0.0f;  // bias gradient: column sums of dZ2 (wave 0 only)
  const int n_items = fl_count(fl, n_frames) * NB;
  // The next item's band is loaded into registers while this one computes (the load and
  // the MFMA phases of the two workgroups on a CU otherwise ran in lockstep, unoverlapped).
  constexpr int NVX = (NX / 4 + 255) / 256, NVD = ((BR * OW + 1) / 2 * 2 * 8 + 255) / 256;
  f4 px4[NVX], pd4[NVD];
  auto load_item = [&](int it) {
    const int f = fl_frame(fl, it / NB), band = it - (it / NB) * NB;
    const int oy0 = BR * band, nr = min(BR, OH - oy0), npb = nr * OW, npe = (npb + 1) / 2 * 2;
    const int y0 = 2 * oy0, nx = min(2 * nr + 2, IH - y0) * IW * 32;
    const f4* s4 = reinterpret_cast<const f4*>(X1 + ((int64_t)f * IH + y0) * IW * 32);
#pragma unroll
    for (int j = 0; j < NVX; ++j) {
      const int i = tid + 256 * j;
      if (i < nx / 4) px4[j] = s4[i];
    }
    const f4* z4 = reinterpret_cast<const f4*>(dZ2 + ((int64_t)f * NP + oy0 * OW) * 32);
#pragma unroll
    for (int j = 0; j < NVD; ++j) {
      const int i = tid + 256 * j;
      if (i < npe * 8) pd4[j] = i < npb * 8 ? z4[i] : f4zero();
    }
  };
  if ((int)blockIdx.x < n_items) load_item(blockIdx.x);
  for (int it = blockIdx.x; it < n_items; it += gridDim.x) {
    const int band = it - (it / NB) * NB;
    const int oy0 = BR * band, nr = min(BR, OH - oy0), npb = nr * OW, npe = (npb + 1) / 2 * 2;
    const int y0 = 2 * oy0, nx = min(2 * nr + 2, IH - y0) * IW * 32;
    {
      f4* d4 = reinterpret_cast<f4*>(xs);
#pragma unroll
      for (int j = 0; j < NVX; ++j) {
        const int i = tid + 256 * j;
        if (i < nx / 4) d4[i] = px4[j];
      }
      f4* e4 = reinterpret_cast<f4*>(ds);
#pragma unroll
      for (int j = 0; j < NVD; ++j) {
        const int i = tid + 256 * j;
        if (i < npe * 8) e4[i] = pd4[j];
      }
    }
    __syncthreads();
    if (it + (int)gridDim.x < n_items) load_item(it + gridDim.x);
#pragma unroll 3
    for (int s = 0; s < npe / 2; ++s) {
      const int p = 2 * s + h;
      const float a = ds[p * 32 + c32];
      if (wave == 0) bacc += a;
      const int pp = p < npb ? p : 0;
      const int oy = pp / OW, ox = pp - (pp / OW) * OW;
      const float* xb = xs + ((2 * oy) * IW + 2 * ox) * 32 + c32;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int tap = wave * 4 + j, ky = tap >> 2, kx = tap & 3;
        acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, xb[(ky * IW + kx) * 32], acc[j], 0, 0, 0);
      }
    }
    __syncthreads();
  }
  float* out = slab + (int64_t)blockIdx.x * (32 * 512);
  if (wave == 0) {
    bacc += __shfl_xor(bacc, 32);
    if (h == 0) bias_slab[(int64_t)blockIdx.x * 32 + c32] = bacc;
  }
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int co = (r & 3) + 8 * (r >> 2) + 4 * h;
      out[co * 512 + (wave * 4 + j) * 32 + c32] = acc[j][r];
    }
}

// ---- conv2 input gradient -------------------------------------------------------
// dX1[f][y][x][ci] = [X1 > 0] * sum over the (ky, kx) taps reaching (y, x) and co of
// dZ2[f][oy][ox][co] * W2[co][ky][kx][ci]  (k4 s2). Wave w owns the input-parity class
// (py, px) = (w >> 1, w & 1): its (KH/S)^2 = 4 taps are fixed, so its 64 B fragments (k =
// tap*32 + co, 16x16x4 MFMA, 2 column tiles of ci) stay in registers for the whole kernel.
// dZ2_f is staged in LDS with one extra zero row that out-of-range taps point at, pixel
// rows padded to 34 floats: the 16 pixels x 2 channel lanes of a ds_read_b32 half then
// fall on distinct banks (2p + q mod 32), where a 32-float stride put all 16 pixels of a
// channel on one bank (SQ_LDS_BANK_CONFLICT 3.4e9 per update before). Maps whose padded
// copy would cost a resident workgroup (174x174: 3 per CU) use 33 (2-way at worst).
// BITS: the ReLU mask comes from conv1's bitmask (one uint32 of channel bits per pixel)
// instead of X1 itself — 4 B instead of 128 B of reads per pixel.
template <int IH, int IW, int OH, int OW, bool BITS>
__global__ __launch_bounds__(256) void conv2_dgrad_kernel(const float* __restrict__ dZ2, const float* __restrict__ WT,
                                                          const float* __restrict__ X1,
                                                          const uint32_t* __restrict__ mask, float* __restrict__ dX1,
                                                          int n_frames) {
  constexpr int NP = OH * OW;
  constexpr int HYC = IH / 2, WXC = IW / 2;  // even input sizes: every class has HYC x WXC pixels
  static_assert(IH % 2 == 0 && IW % 2 == 0, "even conv1 maps");
  constexpr int NPC = HYC * WXC;
  constexpr int TILES = (NPC + 15) / 16;
  constexpr int PS = ((NP + 1) * 34 * 4 <= 160 * 1024 / 3 || (NP + 1) * 33 * 4 > 160 * 1024 / 3) ? 34 : 33;
  __shared__ __attribute__((aligned(16))) float ds[(NP + 1) * PS];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int py = wave >> 1, px = wave & 1;
  const int i16 = lane & 15, q = lane >> 4;
  // B fragments: step s covers k = 4s..4s+3 -> tap = s / 8, co = 4*(s % 8) + q
  float b[32][2];
#pragma unroll
  for (int s = 0; s < 32; ++s) {
    const int tap = s >> 3, co = 4 * (s & 7) + q;
    const int ky = py + 2 * (tap >> 1), kx = px + 2 * (tap & 1);
#pragma unroll
    for (int ct = 0; ct < 2; ++ct) b[s][ct] = WT[((ky * 4 + kx) * 32 + ct * 16 + i16) * 32 + co];
  }
  if (tid < 32) ds[NP * PS + tid] = 0.0f;
  // software pipeline: the next frame's dZ2 is loaded into registers while this one computes
  constexpr int NZ = (NP * 8 + 255) / 256;
  f4 zr[NZ];
  auto load_z = [&](int f) {
    const f4* z4 = reinterpret_cast<const f4*>(dZ2 + (int64_t)f * NP * 32);
#pragma unroll
    for (int j = 0; j < NZ; ++j) {
      const int i = tid + j * 256;
      if (i < NP * 8) zr[j] = z4[i];
    }
  };
  if (blockIdx.x < n_frames) load_z(blockIdx.x);
  for (int f = blockIdx.x; f < n_frames; f += gridDim.x) {
    {
      typedef float f2 __attribute__((ext_vector_type(2)));
#pragma unroll
      for (int j = 0; j < NZ; ++j) {
        const int i = tid + j * 256;
        if (i >= NP * 8) break;
        const f4 v = zr[j];
        float* d = ds + (i >> 3) * PS + 4 * (i & 7);
        if constexpr (PS % 2 == 0) {
          reinterpret_cast<f2*>(d)[0] = f2{v[0], v[1]};
          reinterpret_cast<f2*>(d)[1] = f2{v[2], v[3]};
        } else {
          d[0] = v[0];
          d[1] = v[1];
          d[2] = v[2];
          d[3] = v[3];
        }
      }
    }
    __syncthreads();
    if (f + (int)gridDim.x < n_frames) load_z(f + gridDim.x);
    for (int t = 0; t < TILES; ++t) {
      const int pc = t * 16 + i16;  // this lane's pixel of the class (A row)
      const int yy = pc / WXC, xx = pc - (pc / WXC) * WXC;
      int off[4];
#pragma unroll
      for (int tap = 0; tap < 4; ++tap) {
        const int oy = yy - (tap >> 1), ox = xx - (tap & 1);
        const bool ok = pc < NPC && oy >= 0 && oy < OH && ox >= 0 && ox < OW;
        off[tap] = (ok ? (oy * OW + ox) : NP) * PS + q;
      }
      f4 acc0 = f4zero(), acc1 = f4zero();
#pragma unroll
      for (int s = 0; s < 32; ++s) {
        const float a = ds[off[s >> 3] + 4 * (s & 7)];
        acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b[s][0], acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b[s][1], acc1, 0, 0, 0);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int pr = t * 16 + q * 4 + r;
        if (pr < NPC) {
          const int y = (pr / WXC) * 2 + py, x = (pr % WXC) * 2 + px;
          const int64_t pix = ((int64_t)f * IH + y) * IW + x;
          const int64_t base = pix * 32 + i16;
          if constexpr (BITS) {
            const uint32_t mw = mask[pix];
            dX1[base] = (mw >> i16) & 1u ? acc0[r] : 0.0f;
            dX1[base + 16] = (mw >> (i16 + 16)) & 1u ? acc1[r] : 0.0f;
          } else {
            dX1[base] = X1[base] > 0.0f ? acc0[r] : 0.0f;
            dX1[base + 16] = X1[base + 16] > 0.0f ? acc1[r] : 0.0f;
          }
        }
      }
    }
    __syncthreads();
  }
}

// ---- conv2 input gradient on bf16 MFMA (split operands) ---------------------------
// The same product as conv2_dgrad_kernel with both fp32 operands split by truncation into
// three exact bf16 terms and the six terms of magnitude >= 2^-16 summed on
// v_mfma_f32_16x16x32_bf16 (gemm_x6_kernel's scheme: dropped terms are below fp32 rounding).
// Wave w owns parity class (py, px) = ((w & 3) >> 1, w & 1) (with 8 waves, waves w and w + 4
// take alternate tile pairs of the class); K step t = tap t (32 co), so an A
// fragment (lane: class pixel i16, co 8q..8q+7 of one tap) is one 16-B read of a split dZ2
// plane; dZ2_f is split once when it is staged into three planes. Plane rows: dZ2 pixel
// (oy, ox) sits at row (oy + 1) * WXC + ox + 1 (WXC = IW / 2 = OW + 1), so tap (ty, tx) of
// class pixel pc = yy * WXC + xx reads row pc + (1 - ty) WXC + (1 - tx): the 16 pixels of a
// tile read 16 CONSECUTIVE rows for every tap, and out-of-range taps land on rows no pixel
// owns (the gap column, the rows above and below), zeroed once. Rows are 32 bf16 (4 quads)
// with the quads of row r rotated by 2 (r >> 2): the 4 lane groups of a ds_read_b128 then hit
// 16 distinct bank quads at any tile offset (tools/dgrad_banks.py: 1.09 -> 0 extra cycles per
// group at 174x174; the former 40-bf16 rows with a shared zero row conflicted 2-way). The
// split weights (4 taps x 2 ci tiles x 3 terms) stay in registers; two 16-pixel tiles run
// together (four independent accumulators).
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));

template <int IH, int IW>
constexpr int conv2_dgrad_x6_rows() {  // plane rows: the last tile's reads, padding included
  return ((IH / 2) * (IW / 2) + 15) / 16 * 16 + IW / 2 + 1;
}

template <int IH, int IW, int OH, int OW>
constexpr size_t conv2_dgrad_x6_lds() {  // three dZ2 planes + the frame's conv1 ReLU words
  return (size_t)3 * conv2_dgrad_x6_rows<IH, IW>() * 32 * 2 + (size_t)IH * IW * 4;
}

// bf16 offset of quad q of plane row r of NQ quads (the rotation above; rows of 8 quads, 64
// channels, rotate by r: conflict-free for the same lane groups, tools/dgrad_banks.py)
template <int NQ = 4>
__device__ __forceinline__ int dg_quad_off(int r, int q) {
  static_assert(NQ == 4 || NQ == 8, "rows of 32 or 64 bf16");
  if constexpr (NQ == 4)
    return r * 32 + 8 * ((q + 2 * (r >> 2)) & 3);
  else
    return r * 64 + 8 * ((q + r) & 7);
}

template <int IH, int IW, int OH, int OW>
constexpr bool conv2_dgrad_x6_fits() {
  return IH % 2 == 0 && IW % 2 == 0 && conv2_dgrad_x6_lds<IH, IW, OH, OW>() <= 160 * 1024;
}

// Waves per workgroup: 4 (one per parity class) while two workgroups share a CU's LDS
// (84x84: 20x20 conv1 map, 24 KB of planes); 8 (two per class, alternate tile pairs) when
// the planes take more than half the LDS (174x174: 42x42 map, 96 KB) — the same 2 waves
// per SIMD from one workgroup.
template <int IH, int IW, int OH, int OW>
constexpr int conv2_dgrad_x6_waves() {
  return conv2_dgrad_x6_lds<IH, IW, OH, OW>() <= 64 * 1024 ? 4 : 8;
}

__device__ __forceinline__ void split3_pack(const f4& v, uint2& t0, uint2& t1, uint2& t2) {
  uint16_t h[4], m[4], l[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) split3_bf16(v[e], h[e], m[e], l[e]);
  t0 = uint2{h[0] | ((uint32_t)h[1] << 16), h[2] | ((uint32_t)h[3] << 16)};
  t1 = uint2{m[0] | ((uint32_t)m[1] << 16), m[2] | ((uint32_t)m[3] << 16)};
  t2 = uint2{l[0] | ((uint32_t)l[1] << 16), l[2] | ((uint32_t)l[3] << 16)};
}

// The product is computed transposed (MFMA rows = ci, columns = pixels), so the epilogue
// stores 4 consecutive channels of a pixel per lane straight from the accumulators (16-B
// stores under 4 bits of the conv1 ReLU bitmask: 4x fewer store instructions than the
// pixel-row layout's dword stores, which left the kernel store-issue bound; staging the
// result in LDS instead cost a resident workgroup and measured slower).
//
// ROT (round 6): at 174x174 one 8-wave workgroup fills a CU, and its item loop began with
// s_waitcnt vmcnt(0) — the staging of frame i + 1 waited for frame i's 226 KB of dX1 stores to
// be acknowledged, with no other workgroup to fill the CU meanwhile (the compiler's one wait
// for the first iteration, which has no store in flight, and the later ones). ROT rotates the
// loop (load next, tiles, barrier, stage next, barrier) with a fixed tile-pair count per wave
// and unconditional stores — lanes past the class map store to `sink` — so the staging waits
// for its own loads only (vmcnt(stores + later loads)). Same products, same order: bitwise.
template <int IH, int IW, int OH, int OW, int NW, bool ROT = false>
__global__ __launch_bounds__(NW * 64, 2) void conv2_dgrad_x6_kernel(const float* __restrict__ dZ2,
                                                                const float* __restrict__ WT,
                                                                const uint32_t* __restrict__ mask,
                                                                float* __restrict__ dX1, int n_frames, FrameList fl,
                                                                float* __restrict__ sink) {
  constexpr int NP = OH * OW;
  constexpr int HYC = IH / 2, WXC = IW / 2, NPC = HYC * WXC;
  constexpr int TILES = (NPC + 15) / 16;
  constexpr int NR = conv2_dgrad_x6_rows<IH, IW>();
  constexpr int PL = NR * 32;  // plane size (bf16)
  static_assert(IH % 2 == 0 && IW % 2 == 0, "even conv1 maps");
  static_assert(WXC == OW + 1, "k4 s2: the class width is the dZ2 width + 1 (the gap column)");
  extern __shared__ __attribute__((aligned(16))) uint8_t smem_dg[];
  uint16_t* zs = reinterpret_cast<uint16_t*>(smem_dg);
  // the frame's ReLU words, staged with dZ2: a global load in the epilogue made every tile
  // wait (vmcnt counts stores too) for its previous tile's stores
  uint32_t* ms = reinterpret_cast<uint32_t*>(smem_dg + (size_t)3 * PL * 2);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  constexpr int NT = NW * 64;
  const int cls = wave & 3, py = cls >> 1, px = cls & 1;
  const int i16 = lane & 15, q = lane >> 4;
  bf16x8_t bw[4][2][3];  // [tap][ci tile][term]: B[k = co 8q + j][ci]
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int ky = py + 2 * (t >> 1), kx = px + 2 * (t & 1);
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) {
      union { uint16_t u[8]; bf16x8_t v; } b0, b1, b2;
#pragma unroll
      for (int j = 0; j < 8; ++j)
        split3_bf16(WT[((ky * 4 + kx) * 32 + nt * 16 + i16) * 32 + 8 * q + j], b0.u[j], b1.u[j], b2.u[j]);
      bw[t][nt][0] = b0.v;
      bw[t][nt][1] = b1.v;
      bw[t][nt][2] = b2.v;
    }
  }
  // every plane row zero once: rows no dZ2 pixel owns stay zero (the staging writes only the
  // pixels' rows), the barrier orders these stores before the first frame's
  for (int i = tid; i < 3 * PL / 8; i += NT) reinterpret_cast<uint4*>(zs)[i] = uint4{0u, 0u, 0u, 0u};
  __syncthreads();
  constexpr int NZ = (NP * 8 + NT - 1) / NT, NM = (IH * IW + NT - 1) / NT;
  f4 zr[NZ];
  uint32_t mr[NM];
  // staging slot i -> (pixel i >> 3, 4-channel chunk i & 7), pixel-major (coalesced 128-B
  // dZ2 runs): two neighbouring pixels' 8-B writes fill a 16-lane group's 32 banks once
  auto slot_pc = [](int i) { return i; };
  // dZ2 and the ReLU words of frame f, into registers; unconditional (slots past the frame
  // reload its last one, staging skips them; past the last frame the frame repeats): no branch
  // around the loads for the compiler's wait counts to get lost in
  // item i (list position) -> frame fl_frame(fl, i)
  auto load_z = [&](int i) {
    const int f = fl_frame(fl, i);
    const f4* z4 = reinterpret_cast<const f4*>(dZ2 + (int64_t)f * NP * 32);
#pragma unroll
    for (int j = 0; j < NZ; ++j) zr[j] = z4[min(slot_pc(tid + j * NT), NP * 8 - 1)];
#pragma unroll
    for (int j = 0; j < NM; ++j) mr[j] = mask[(int64_t)f * IH * IW + min(tid + j * NT, IH * IW - 1)];
  };
  auto stage = [&]() {
#pragma unroll
    for (int j = 0; j < NZ; ++j) {
      const int i = slot_pc(tid + j * NT);
      if (i < NP * 8) {
        uint2 t0, t1, t2;
        split3_pack(zr[j], t0, t1, t2);
        const int p = i >> 3, c = i & 7;
        uint16_t* d = zs + dg_quad_off(p + p / OW + WXC + 1, c >> 1) + 4 * (c & 1);
        *reinterpret_cast<uint2*>(d) = t0;
        *reinterpret_cast<uint2*>(d + PL) = t1;
        *reinterpret_cast<uint2*>(d + 2 * PL) = t2;
      }
    }
#pragma unroll
    for (int j = 0; j < NM; ++j) {
      const int i = tid + j * NT;
      if (i < IH * IW) ms[i] = mr[j];
    }
  };
  n_frames = fl_count(fl, n_frames);
  if ((int)blockIdx.x < n_frames) {
    load_z(blockIdx.x);
    if constexpr (ROT) stage();
  }
  if constexpr (ROT) __syncthreads();
  // tile pairs per wave: t0 = 2 (wave >> 2) + 2 (NW / 4) k (84x84: 4, 174x174: 7)
  constexpr int NIT = (TILES + 2 * (NW / 4) - 1) / (2 * (NW / 4));
  for (int fi = blockIdx.x; fi < n_frames; fi += gridDim.x) {
    const int f = fl_frame(fl, fi);
    if constexpr (!ROT) {
      stage();
      __syncthreads();
    }
    load_z(min(fi + (int)gridDim.x, n_frames - 1));
    auto tile_pair = [&](int t0) {
      int off[2][4];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int pc = (t0 + u) * 16 + i16;  // this lane's class pixel (A row); past NPC: a row
                                             // the last tile reads, its column never stored
#pragma unroll
        for (int tap = 0; tap < 4; ++tap) off[u][tap] = dg_quad_off(pc + (1 - (tap >> 1)) * WXC + (1 - (tap & 1)), q);
      }
      f4 acc[2][2];
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) acc[u][nt] = f4zero();
#pragma unroll
      for (int tap = 0; tap < 4; ++tap) {
        bf16x8_t a[2][3];
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
          for (int tm = 0; tm < 3; ++tm) a[u][tm] = *reinterpret_cast<const bf16x8_t*>(zs + tm * PL + off[u][tap]);
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
          for (int nt = 0; nt < 2; ++nt) {  // small terms first; D^T = W^T dZ2^T: rows = ci, cols = pixels
            f4 c = acc[u][nt];
            c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bw[tap][nt][0], a[u][2], c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bw[tap][nt][2], a[u][0], c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bw[tap][nt][1], a[u][1], c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bw[tap][nt][0], a[u][1], c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bw[tap][nt][1], a[u][0], c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bw[tap][nt][0], a[u][0], c, 0, 0, 0);
            acc[u][nt] = c;
          }
      }
      // the transposed product leaves lane (pixel i16, q) holding channels nt*16 + 4q .. +3 of
      // its pixel: one 16-B store per (tile, ci tile) under 4 bits of the ReLU mask
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int pr = (t0 + u) * 16 + i16;
        if (ROT) {  // unconditional: a lane past the class map stores to the sink
          const int pv = min(pr, NPC - 1);
          const int y = (pv / WXC) * 2 + py, x = (pv % WXC) * 2 + px;
          const int64_t pix = ((int64_t)f * IH + y) * IW + x;
          const uint32_t mw = ms[y * IW + x];
#pragma unroll
          for (int nt = 0; nt < 2; ++nt) {
            const uint32_t m4 = mw >> (nt * 16 + 4 * q);
            f4 v = acc[u][nt];
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] = (m4 >> r) & 1u ? v[r] : 0.0f;
            *reinterpret_cast<f4*>(pr < NPC ? dX1 + pix * 32 + nt * 16 + 4 * q : sink) = v;
          }
        } else if (pr < NPC) {
          const int y = (pr / WXC) * 2 + py, x = (pr % WXC) * 2 + px;
          const int64_t pix = ((int64_t)f * IH + y) * IW + x;
          const uint32_t mw = ms[y * IW + x];
#pragma unroll
          for (int nt = 0; nt < 2; ++nt) {
            const uint32_t m4 = mw >> (nt * 16 + 4 * q);
            f4 v = acc[u][nt];
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] = (m4 >> r) & 1u ? v[r] : 0.0f;
            *reinterpret_cast<f4*>(dX1 + pix * 32 + nt * 16 + 4 * q) = v;
          }
        }
      }
    };
    if constexpr (ROT) {
#pragma unroll 1
      for (int k = 0; k < NIT; ++k) tile_pair(2 * (wave >> 2) + 2 * (NW / 4) * k);
      __syncthreads();  // every wave done with this frame's planes and ReLU words
      stage();          // the next frame's (past the last one: the last one again)
    } else {
#pragma unroll 1
      for (int t0 = 2 * (wave >> 2); t0 < TILES; t0 += 2 * (NW / 4)) tile_pair(t0);
    }
    __syncthreads();
  }
}

// ---- conv2 input gradient, banded (maps too large to stage whole: 300x400) ------------
// The product of conv2_dgrad_x6_kernel over a band of BY rows of the conv1 map: a work item is
// (frame, band); the dZ2 rows its pixels' taps reach (BY/2 + 1 of them) are split once into
// three bf16 planes, the band's conv1 ReLU words staged beside them, the next item's rows
// prefetched into registers. Wave w owns parity class (py, px) = (w >> 1, w & 1) with its
// split weights in registers; a class's width is (IW - px + 1) / 2, so odd maps (99 columns)
// work. Plane rows as in the whole-map kernel, with one row pitch WX = (IW + 1) / 2 for both
// classes (the narrower class's last column is a dummy: computed, not stored): staged dZ2 row
// j (oy = zlo + j) in row block j + 1, pixel ox at column ox + 1, so class pixel (yl, xx) of the
// band reads row (yl + yy0 - zlo + 1 - ty) WX + xx + 1 - tx, consecutive along a 16-pixel tile;
// block 0 and the gap columns are never written (zero), the blocks past a short last band's
// rows are zeroed per item; quads rotated (dg_quad_off): conflict-free reads
// (tools/dgrad_banks.py). 74x99 conv1 map, BY = 8: 74 KB of LDS, two workgroups per CU; dZ2 is
// staged 1.25x (a row shared by neighbouring bands).
constexpr int conv2_dgband_rows(int IW, int BY) {  // plane rows: BY/2 + 3 blocks of WX, + a tile's overhang
  return (BY / 2 + 3) * ((IW + 1) / 2) + 16;
}
constexpr size_t conv2_dgband_lds(int IW, int OW, int BY) {  // 3 planes, ReLU words
  return (size_t)3 * conv2_dgband_rows(IW, BY) * 32 * 2 + (size_t)BY * IW * 4 + 0 * OW;
}

template <int IH, int IW, int OH, int OW, int BY>
struct Conv2DgBand {
  static_assert(BY % 2 == 0, "bands of whole parity rows");
  static constexpr int NB = (IH + BY - 1) / BY;  // bands per frame
  static constexpr int ZR = BY / 2 + 1;          // staged dZ2 rows
  static constexpr int WX = (IW + 1) / 2;        // row pitch of both classes
  static constexpr int NR = conv2_dgband_rows(IW, BY);
  static constexpr int PL = NR * 32;             // plane size (bf16)
  static constexpr size_t LDS = conv2_dgband_lds(IW, OW, BY);
  static_assert(WX >= OW + 1, "a gap column left of every dZ2 row");
};

template <int IW, int OW>
constexpr int conv2_dgrad_band_rows() {  // the largest even band whose LDS keeps 2 workgroups per CU
  int by = 16;
  while (by > 2 && conv2_dgband_lds(IW, OW, by) > 80 * 1024) by -= 2;
  return by;
}

template <int IH, int IW, int OH, int OW, int BY>
__global__ __launch_bounds__(256, 2) void conv2_dgrad_band_x6_kernel(const float* __restrict__ dZ2,
                                                                     const float* __restrict__ WT,
                                                                     const uint32_t* __restrict__ mask,
                                                                     float* __restrict__ dX1, int n_frames,
                                                                     FrameList fl) {
  using B = Conv2DgBand<IH, IW, OH, OW, BY>;
  constexpr int NB = B::NB, ZR = B::ZR, WX = B::WX, PL = B::PL, NT = 256;
  constexpr int NP = OH * OW;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem_db[];
  uint16_t* zs = reinterpret_cast<uint16_t*>(smem_db);
  uint32_t* ms = reinterpret_cast<uint32_t*>(smem_db + (size_t)3 * PL * 2);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int py = wave >> 1, px = wave & 1;
  const int xc = (IW - px + 1) / 2;  // class width
  const int i16 = lane & 15, q = lane >> 4;
  bf16x8_t bw[4][2][3];  // [tap][ci tile][term]: B[k = co 8q + j][ci]
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int ky = py + 2 * (t >> 1), kx = px + 2 * (t & 1);
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) {
      union { uint16_t u[8]; bf16x8_t v; } b0, b1, b2;
#pragma unroll
      for (int j = 0; j < 8; ++j)
        split3_bf16(WT[((ky * 4 + kx) * 32 + nt * 16 + i16) * 32 + 8 * q + j], b0.u[j], b1.u[j], b2.u[j]);
      bw[t][nt][0] = b0.v;
      bw[t][nt][1] = b1.v;
      bw[t][nt][2] = b2.v;
    }
  }
  // every plane row zero once (block 0, the gap columns); the barrier orders these stores
  // before the first item's
  for (int i = tid; i < 3 * PL / 8; i += NT) reinterpret_cast<uint4*>(zs)[i] = uint4{0u, 0u, 0u, 0u};
  __syncthreads();
  constexpr int NZ = (ZR * OW * 8 + NT - 1) / NT, NM = (BY * IW + NT - 1) / NT;
  f4 zr[NZ];
  uint32_t mr[NM];
  auto z_lo = [](int band) { return max(BY / 2 * band - 1, 0); };
  auto z_rows = [&](int band) { return min(BY / 2 * band + BY / 2, OH) - z_lo(band); };
  auto b_rows = [](int band) { return min(BY, IH - BY * band); };
  // item it = (list item it / NB, band it % NB): its dZ2 rows and ReLU words into registers,
  // unconditional (clamped: slots past the band reload its last one; staging skips them)
  auto load = [&](int it) {
    const int f = fl_frame(fl, it / NB), band = it - (it / NB) * NB;
    const int nz = z_rows(band) * OW * 8, nm = b_rows(band) * IW;
    const f4* z4 = reinterpret_cast<const f4*>(dZ2 + ((int64_t)f * OH + z_lo(band)) * OW * 32);
#pragma unroll
    for (int j = 0; j < NZ; ++j) zr[j] = z4[min(tid + j * NT, nz - 1)];
    const uint32_t* m = mask + ((int64_t)f * IH + BY * band) * IW;
#pragma unroll
    for (int j = 0; j < NM; ++j) mr[j] = m[min(tid + j * NT, nm - 1)];
  };
  const int n_items = fl_count(fl, n_frames) * NB;
  if ((int)blockIdx.x < n_items) load(blockIdx.x);
  for (int it = blockIdx.x; it < n_items; it += gridDim.x) {
    const int f = fl_frame(fl, it / NB), band = it - (it / NB) * NB;
    const int zlo = z_lo(band), nzr = z_rows(band), nz = nzr * OW * 8, by = b_rows(band);
    if (nzr < ZR && band > 0) {  // a short last band: its taps past the map read blocks nzr + 1 .. ZR
      const int r0 = (nzr + 1) * WX, nw = (ZR - nzr) * WX * 32 / 8;  // 16-B words per plane
      for (int i = tid; i < 3 * nw; i += NT) {
        const int pl = i / nw;
        reinterpret_cast<uint4*>(zs + pl * PL + r0 * 32)[i - pl * nw] = uint4{0u, 0u, 0u, 0u};
      }
    }
#pragma unroll
    for (int j = 0; j < NZ; ++j) {
      const int i = tid + j * NT;
      if (i < nz) {
        uint2 t0, t1, t2;
        split3_pack(zr[j], t0, t1, t2);
        const int p = i >> 3, c = i & 7;
        uint16_t* d = zs + dg_quad_off((p / OW + 1) * WX + p % OW + 1, c >> 1) + 4 * (c & 1);
        *reinterpret_cast<uint2*>(d) = t0;
        *reinterpret_cast<uint2*>(d + PL) = t1;
        *reinterpret_cast<uint2*>(d + 2 * PL) = t2;
      }
    }
#pragma unroll
    for (int j = 0; j < NM; ++j) {
      const int i = tid + j * NT;
      if (i < by * IW) ms[i] = mr[j];
    }
    __syncthreads();
    load(min(it + (int)gridDim.x, n_items - 1));
    const int yy0 = BY / 2 * band;             // first class row of the band (both py: y0 even)
    const int ncy = (by - py + 1) / 2;         // class rows of this class in the band
    const int npc = ncy * WX, tiles = (npc + 15) / 16;
    const int rb = (yy0 - zlo + 1) * WX + 1;   // plane row of class pixel 0 at tap (0, 0)
#pragma unroll 1
    for (int t0 = 0; t0 < tiles; t0 += 2) {
      int off[2][4];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int pc = (t0 + u) * 16 + i16;  // this lane's class pixel (A row), pitch WX
#pragma unroll
        for (int tap = 0; tap < 4; ++tap) off[u][tap] = dg_quad_off(pc + rb - (tap >> 1) * WX - (tap & 1), q);
      }
      f4 acc[2][2];
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) acc[u][nt] = f4zero();
#pragma unroll
      for (int tap = 0; tap < 4; ++tap) {
        bf16x8_t a[2][3];
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
          for (int tm = 0; tm < 3; ++tm) a[u][tm] = *reinterpret_cast<const bf16x8_t*>(zs + tm * PL + off[u][tap]);
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
          for (int nt = 0; nt < 2; ++nt) {  // small terms first (conv2_dgrad_x6_kernel's order)
            f4 c = acc[u][nt];
            c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bw[tap][nt][0], a[u][2], c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bw[tap][nt][2], a[u][0], c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bw[tap][nt][1], a[u][1], c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bw[tap][nt][0], a[u][1], c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bw[tap][nt][1], a[u][0], c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bw[tap][nt][0], a[u][0], c, 0, 0, 0);
            acc[u][nt] = c;
          }
      }
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int pc = (t0 + u) * 16 + i16;
        const int yl = pc / WX, xx = pc - (pc / WX) * WX;
        if (pc < npc && xx < xc) {
          const int y = 2 * (yy0 + yl) + py, x = 2 * xx + px;
          const int64_t pix = ((int64_t)f * IH + y) * IW + x;
          const uint32_t mw = ms[(y - BY * band) * IW + x];
#pragma unroll
          for (int nt = 0; nt < 2; ++nt) {
            const uint32_t m4 = mw >> (nt * 16 + 4 * q);
            f4 v = acc[u][nt];
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] = (m4 >> r) & 1u ? v[r] : 0.0f;
            *reinterpret_cast<f4*>(dX1 + pix * 32 + nt * 16 + 4 * q) = v;
          }
        }
      }
    }
    __syncthreads();
  }
  (void)NP;
}

// ---- conv2 forward on bf16 MFMA (split operands) -----------------------------------
// X2[f][oy][ox][co] = relu(b[co] + sum over taps (ky, kx) and ci of
// X1[f][2oy+ky][2ox+kx][ci] * W2[co][ky][kx][ci])  (k4 s2, 32 -> 32 channels).
// Work item = (frame, band of BR output rows); 8 waves: wave w owns kernel row ky = w & 3
// (taps (ky, 0..3), their split weights — 4 taps x 2 co tiles x 3 terms — in registers) and
// the pixel tiles t = w >> 2 (mod 2) of the band. The band's X1 rows are split once when they
// are staged, into three bf16 planes laid out [row][x & 1][x >> 1][ci] (pixel stride 40:
// the 16 pixels of a B fragment — consecutive ox, stride-2 x — fall on distinct bank quads),
// so each x6 product reads its operands with one ds_read_b128 per term instead of gathering
// and splitting an im2col tile per K step from L2 (the generic path's VALU-bound split).
// Each wave's product is D[co][pixel] over its 4 taps (K = 128) on
// v_mfma_f32_16x16x32_bf16; the four kernel-row partials go to LDS and are summed in a
// fixed order with the bias and ReLU, 16 B per thread.
template <int IH, int IW, int OH, int OW>
struct Conv2FwdBand {
  static constexpr int WH = (IW + 1) / 2;  // x >> 1 columns per parity
  // 84x84 (20x20 -> 9x9, one band): tiles of 2 rows x 8 pixels plus the last row and column
  // (pix2x8 below) on unpadded pixels, the odd-x plane 4 quads past the even one and rows 1 quad
  // apart: 1/8 of the B-fragment read conflict cycles of the row-major tiles at pixel stride 40
  // and conflict-free split stores (exhaustive check: tools/conv2f84_banks.py)
  static constexpr bool kTiled = IH == 20 && IW == 20 && OH == 9 && OW == 9;
  // other maps: unpadded pixels (4 quads of 8 channels), quad q of parity column xh stored at
  // slot (q + (xh >> 1)) & 3 — the 16 pixels of a B fragment (consecutive ox) then sit on 16
  // distinct bank quads in each ds_read_b128 lane group, where the former 5-quad pixel stride
  // conflicted 2-way in every group (tools/conv2f_banks.py; 0.46 of the LDS cycles at 300x400)
  static constexpr int PSX = 32;                            // pixel stride in a plane (bf16)
  static constexpr int PO = kTiled ? 352 : WH * PSX;        // odd-x plane offset (bf16)
  static constexpr int RSP = kTiled ? 680 : 2 * WH * PSX;   // plane row stride (bf16)
  static constexpr int rows_of(int br) { return 2 * br + 2 < IH ? 2 * br + 2 : IH; }
  static constexpr int tiles_of(int br) { return (br * OW + 15) / 16; }
  static constexpr size_t planes_of(int br) { return (size_t)3 * rows_of(br) * RSP * 2; }
  // partial sums [4 kernel rows][band pixels][PP]: rows padded to 36 floats so the 16 pixels
  // of an MFMA tile's f4 stores land on distinct bank quads (32: 8-way conflicts)
  static constexpr int PP = 36;
  static constexpr size_t lds_of(int br) { return planes_of(br) + (size_t)4 * tiles_of(br) * 16 * PP * 4; }
  static constexpr int br_max() {
    int br = OH;
    while (br > 1 && lds_of(br) > 160 * 1024) --br;
    return br;
  }
  static constexpr int NB = (OH + br_max() - 1) / br_max();
  static constexpr int BR = (OH + NB - 1) / NB;
  static constexpr size_t LDS = lds_of(BR);
};

// Whole frames only: banded maps (174x174, 300x400) re-stage overlapping X1 rows and, at one
// workgroup per CU, measured slower than the generic im2col GEMM (1.09 vs 0.97 ms per 174x174
// rollout step); the 20x20 map of 84x84 frames runs 179 vs 212 us.
template <int IH, int IW, int OH, int OW>
constexpr bool conv2_fwd_x6_fits() {
  return Conv2FwdBand<IH, IW, OH, OW>::NB == 1 && Conv2FwdBand<IH, IW, OH, OW>::LDS <= 160 * 1024;
}

template <int IH, int IW, int OH, int OW>
__global__ __launch_bounds__(512, 2) void conv2_fwd_x6_kernel(const float* __restrict__ X1,
                                                              const float* __restrict__ W2,
                                                              const float* __restrict__ bias,
                                                              float* __restrict__ X2, int n_frames, FrameList fl) {
  using Bd = Conv2FwdBand<IH, IW, OH, OW>;
  constexpr int BR = Bd::BR, NB = Bd::NB, PSX = Bd::PSX, RSP = Bd::RSP, PO = Bd::PO;
  constexpr bool kTiled = Bd::kTiled;
  static_assert(!kTiled || (NB == 1 && Bd::tiles_of(BR) == 6), "tiled 9x9 map");
  // tile pixel of slot (t, i) for the 9x9 map: tiles 0-3 = rows 2t, 2t+1 x ox 0-7, tile 4 = row
  // 8 x ox 0-7 then column 8 x rows 0-7, tile 5 = (8, 8) in every lane; and back
  auto pix2x8 = [](int t, int i, int& oy, int& ox) {
    if (t < 4) {
      oy = 2 * t + (i >> 3);
      ox = i & 7;
    } else if (t == 4) {
      oy = i < 8 ? 8 : i - 8;
      ox = i < 8 ? i : 8;
    } else {
      oy = 8;
      ox = 8;
    }
  };
  auto slot2x8 = [](int oy, int ox) {
    return ox < 8 ? (oy < 8 ? (oy >> 1) * 16 + (oy & 1) * 8 + ox : 64 + ox) : (oy < 8 ? 72 + oy : 80);
  };
  constexpr int BRI = Bd::rows_of(BR), TP = Bd::tiles_of(BR) * 16;  // staged rows, padded band pixels
  constexpr int PL = BRI * RSP;                                        // plane size (bf16)
  constexpr int NP = OH * OW;
  constexpr int NV = (BRI * IW * 8 + 511) / 512;                       // prefetched f4 per thread
  extern __shared__ __attribute__((aligned(16))) uint8_t smem_c2[];
  uint16_t* xs = reinterpret_cast<uint16_t*>(smem_c2);
  float* part = reinterpret_cast<float*>(smem_c2 + (size_t)3 * PL * 2);  // [4][TP][PP]
  constexpr int PP = Bd::PP;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int ky = wave & 3, ph = wave >> 2;
  const int i16 = lane & 15, q = lane >> 4;
  bf16x8_t wf[4][2][3];  // [kx][co tile][term]: A[co = nt*16 + i16][k = ci 8q .. 8q+7]
#pragma unroll
  for (int kx = 0; kx < 4; ++kx)
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) {
      union { uint16_t u[8]; bf16x8_t v; } t0, t1, t2;
      const float* wp = W2 + (nt * 16 + i16) * 512 + (ky * 4 + kx) * 32 + 8 * q;
#pragma unroll
      for (int j = 0; j < 8; ++j) split3_bf16(wp[j], t0.u[j], t1.u[j], t2.u[j]);
      wf[kx][nt][0] = t0.v;
      wf[kx][nt][1] = t1.v;
      wf[kx][nt][2] = t2.v;
    }
  // the bias of this thread's channel quad (c4 = tid & 7 in every reduce iteration), waited for
  // here: a first use inside the loop would wait on the item prefetches in flight as well
  const f4 b4 = *reinterpret_cast<const f4*>(bias + 4 * (tid & 7));
  asm volatile("" ::"v"(b4[0]), "v"(b4[1]), "v"(b4[2]), "v"(b4[3]));
  const int n_items = fl_count(fl, n_frames) * NB;
  auto band_f4 = [&](int band) { return min(BRI, IH - 2 * BR * band) * IW * 8; };
  // two items' X1 in flight: item it + 2 * gridDim.x is loaded into the registers item it
  // just split into LDS (one item of MFMA work was shorter than the load under full load)
  f4 pre[2][NV];
  // staging slot -> band f4 (pixel 8 px + channel quad c4). Untiled maps: within each block of
  // 16 pixels, 16-lane group g stores pixels p0 and p0 + 2 (p0 = 0, 1, 4, 5, ..., 13) — same
  // parity, neighbouring columns: 32 consecutive dwords of one ds_write_b64 group (pixels px and
  // px + 1 sit in different parity planes and overlapped 2-way; tools/conv2f_banks.py)
  auto slot_f4 = [](int i) {
    if constexpr (kTiled) {
      return i;
    } else {
      const int r = i & 127, g = r >> 4;
      return (i & ~127) + 8 * ((g >> 1) * 4 + (g & 1) + 2 * ((r >> 3) & 1)) + (r & 7);
    }
  };
  auto load_item = [&](f4 (&pr)[NV], int it) {
    const int f = fl_frame(fl, it / NB), band = it - (it / NB) * NB;
    const f4* s4 = reinterpret_cast<const f4*>(X1 + ((int64_t)f * IH + 2 * BR * band) * IW * 32);
    const int nv = band_f4(band);
#pragma unroll
    for (int j = 0; j < NV; ++j) pr[j] = s4[min(slot_f4(tid + j * 512), nv - 1)];  // unconditional: countable
  };
  if ((int)blockIdx.x < n_items) load_item(pre[0], blockIdx.x);
  if ((int)(blockIdx.x + gridDim.x) < n_items) load_item(pre[1], blockIdx.x + gridDim.x);
  auto item = [&](auto stage, int it) {
    constexpr int S = decltype(stage)::value;
    const int f = fl_frame(fl, it / NB), band = it - (it / NB) * NB;
    const int oy0 = BR * band, nr = min(BR, OH - oy0), npb = nr * OW;
    {  // split the band's X1 rows into the three planes
      const int nv = band_f4(band);
#pragma unroll
      for (int j = 0; j < NV; ++j) {
        const int i = slot_f4(tid + j * 512);  // a permutation of each 128-slot block
        if (i < nv) {
          const int c4 = i & 7, px = i >> 3, y = px / IW, x = px - (px / IW) * IW;
          uint2 t0, t1, t2;
          split3_pack(pre[S][j], t0, t1, t2);
          const int xh = x >> 1;
          const int qs = kTiled ? (c4 >> 1) : (((c4 >> 1) + (xh >> 1)) & 3);  // the quad's slot
          uint16_t* d = xs + y * RSP + (x & 1) * PO + xh * PSX + 8 * qs + 4 * (c4 & 1);
          *reinterpret_cast<uint2*>(d) = t0;
          *reinterpret_cast<uint2*>(d + PL) = t1;
          *reinterpret_cast<uint2*>(d + 2 * PL) = t2;
        }
      }
    }
    __syncthreads();
    // (a repeat of the last item past the end: unconditional loads keep the wait counts exact)
    load_item(pre[S], min(it + 2 * (int)gridDim.x, n_items - 1));
    const int tiles = (npb + 15) / 16;
    for (int t = ph; t < tiles; t += 2) {
      int oy, ox;
      if constexpr (kTiled) {
        pix2x8(t, i16, oy, ox);
      } else {
        const int p = min(t * 16 + i16, npb - 1);  // this lane's band pixel (B column)
        oy = p / OW;
        ox = p - (p / OW) * OW;
      }
      const uint16_t* xb = xs + (2 * oy + ky) * RSP;
      f4 acc[2] = {f4zero(), f4zero()};
#pragma unroll
      for (int kx = 0; kx < 4; ++kx) {
        const int xh = ox + (kx >> 1);  // tap kx reads x = 2 ox + kx: parity kx & 1, column xh
        const int qs = kTiled ? q : ((q + (xh >> 1)) & 3);
        const uint16_t* xp = xb + (kx & 1) * PO + xh * PSX + 8 * qs;
        bf16x8_t b[3];
#pragma unroll
        for (int tm = 0; tm < 3; ++tm) b[tm] = *reinterpret_cast<const bf16x8_t*>(xp + tm * PL);
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) {  // small terms first
          f4 c = acc[nt];
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[kx][nt][2], b[0], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[kx][nt][0], b[2], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[kx][nt][1], b[1], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[kx][nt][1], b[0], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[kx][nt][0], b[1], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[kx][nt][0], b[0], c, 0, 0, 0);
          acc[nt] = c;
        }
      }
      // lane (pixel i16, q) holds co nt*16 + 4q .. +3 of its pixel
#pragma unroll
      for (int nt = 0; nt < 2; ++nt)
        *reinterpret_cast<f4*>(part + ((ky * TP + t * 16 + i16) * PP + nt * 16 + 4 * q)) = acc[nt];
    }
    __syncthreads();
    const int64_t out0 = ((int64_t)f * NP + oy0 * OW) * 32;
    for (int i = tid; i < npb * 8; i += 512) {  // (pixel, co quad): fixed-order sum of the 4 rows
      const int p = i >> 3, c4 = i & 7;
      const int sl = kTiled ? slot2x8(p / OW, p - (p / OW) * OW) : p;  // the pixel's tile slot
      const f4* pp = reinterpret_cast<const f4*>(part + sl * PP) + c4;
      constexpr int RS4 = TP * PP / 4;  // one kernel row's partials, in f4
      f4 v = ((pp[0] + pp[RS4]) + pp[2 * RS4]) + pp[3 * RS4];
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = fmaxf(v[r] + b4[r], 0.0f);
      *reinterpret_cast<f4*>(X2 + out0 + (int64_t)i * 4) = v;
    }
  };
  for (int it = blockIdx.x; it < n_items; it += 2 * gridDim.x) {
    item(std::integral_constant<int, 0>{}, it);
    if (it + (int)gridDim.x < n_items) item(std::integral_constant<int, 1>{}, it + gridDim.x);
  }
}

// ---- conv2 forward, 42x42 -> 20x20 maps (174x174 frames): one frame streamed per workgroup --
// The banded kernel above re-stages the two X1 rows shared by neighbouring bands and holds a
// 4-way partial sum per pixel; at one 147 KB workgroup per CU it ran no faster than the generic
// im2col product (whose A operand is re-split at each of its 4 uses). This kernel walks the
// bands of a frame in order and keeps the X1 rows in a 14-slot LDS ring (split once into three
// bf16 planes [slot][x & 1][x >> 1][ci], pixel stride 40 as above): band b (output rows 3b ..
// 3b+2) reads X1 rows 6b .. 6b+7, of which only 6 are new (8 for a frame's first band, 4 for its
// last), so every X1 value is loaded from HBM and split exactly once. Slot = row mod 14: the
// rows of band b and the new rows of band b+1 never share a slot, also across a frame boundary
// (42 = 3 x 14). Wave w has role (co tile ct = w & 1, kernel-row half kh = (w >> 1) & 1) with
// its 8 taps' split weights in registers (96 VGPRs), and pixel tiles {w >> 2, (w >> 2) + 2} of
// the band (<= 64 pixels = 4 tiles of 16). The kh = 1 wave of a (ct, tile) writes its partial
// sum to LDS (double-buffered by band parity), the kh = 0 wave adds it to its own after the
// band's barrier, then bias + ReLU and a 16-B store per lane. Schedule per band b, per wave:
// MFMA(b) -> partial(b) -> split of band b+1's rows (prefetched into registers two bands ahead)
// -> loads of band b+3's rows -> barrier -> epilogue(b); one barrier per band, and a wave's
// split runs under the other wave's MFMAs on its SIMD.
struct Conv2Ring42 {
  static constexpr int IH = 42, IW = 42, OH = 20, OW = 20, BR = 3, NB = 7, SLOTS = 14;
  static constexpr int WH = 21, PSX = 32, RSP = 2 * WH * PSX;  // plane row stride (bf16), unpadded
  static constexpr int PL = SLOTS * RSP;                       // plane size (bf16)
  static constexpr int TP = 64, PP = 36;                       // padded band pixels; partial row (floats)
  static constexpr int NV = (8 * IW * 8 + 511) / 512;          // prefetched f4 per thread (<= 8 new rows)
  static constexpr size_t LDS = (size_t)3 * PL * 2 + (size_t)2 * TP * PP * 4;
  static_assert(IH % SLOTS == 0 && LDS <= 160 * 1024, "ring geometry");
  __host__ __device__ static constexpr int new_lo(int b) { return b == 0 ? 0 : 2 * BR * b + 2; }
  __host__ __device__ static constexpr int new_hi(int b) { return 2 * BR * b + 2 * BR + 2 < IH ? 2 * BR * b + 2 * BR + 2 : IH; }
  // 16-B chunk swizzle of X1 row y, plane column xi: chunk q of a pixel is stored at q ^ swz.
  // With the band's tiles (rows 0-2 at ox 0-15, then ox 16-19 of all rows) every 16-lane group
  // of a B-fragment ds_read_b128 and of the split's ds_write_b64 lands on distinct banks
  // (exhaustive check over bands, taps and tiles in tools/ring_banks.py).
  __device__ static int swz(int y, int xi) { return 2 * (((xi >> 2) ^ (y >> 1)) & 1); }
};

template <int IH, int IW, int OH, int OW>
constexpr bool conv2_fwd_ring_fits() {
  return IH == 42 && IW == 42 && OH == 20 && OW == 20;
}

__global__ __launch_bounds__(512, 1) void conv2_fwd_ring_kernel(const float* __restrict__ X1,
                                                                const float* __restrict__ W2,
                                                                const float* __restrict__ bias,
                                                                float* __restrict__ X2, int n_frames, FrameList fl) {
  using R = Conv2Ring42;
  constexpr int IW = R::IW, OW = R::OW, NB = R::NB, WH = R::WH, PSX = R::PSX, RSP = R::RSP, PL = R::PL;
  constexpr int NV = R::NV, PP = R::PP, TP = R::TP, NP = R::OH * R::OW;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem_r2[];
  uint16_t* xs = reinterpret_cast<uint16_t*>(smem_r2);
  float* part = reinterpret_cast<float*>(smem_r2 + (size_t)3 * PL * 2);  // [2][TP][PP]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int ct = wave & 1, kh = (wave >> 1) & 1, tsel = wave >> 2;
  const int i16 = lane & 15, q = lane >> 4;
  bf16x8_t wf[8][3];  // [tap i: ky = 2kh + (i >> 2), kx = i & 3][term]: A[co = ct*16 + i16][k = ci 8q .. 8q+7]
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    union { uint16_t u[8]; bf16x8_t v; } t0, t1, t2;
    const float* wp = W2 + (ct * 16 + i16) * 512 + ((2 * kh + (i >> 2)) * 4 + (i & 3)) * 32 + 8 * q;
#pragma unroll
    for (int j = 0; j < 8; ++j) split3_bf16(wp[j], t0.u[j], t1.u[j], t2.u[j]);
    wf[i][0] = t0.v;
    wf[i][1] = t1.v;
    wf[i][2] = t2.v;
  }
  const f4 b4 = *reinterpret_cast<const f4*>(bias + ct * 16 + 4 * q);
  // make the bias land here: its first use sits in the loop's epilogue, where the compiler
  // cannot tell it from the band prefetches in flight and would wait for vmcnt(0)
  asm volatile("" ::"v"(b4[0]), "v"(b4[1]), "v"(b4[2]), "v"(b4[3]));
  // this workgroup's items: k -> (frame of list item blockIdx.x + (k / NB) * gridDim.x, band k % NB)
  n_frames = fl_count(fl, n_frames);
  const int my_frames = (int)blockIdx.x < n_frames ? (n_frames - 1 - (int)blockIdx.x) / (int)gridDim.x + 1 : 0;
  const int n_items = my_frames * NB;
  auto frame_of = [&](int k) { return fl_frame(fl, (int)blockIdx.x + (k / NB) * (int)gridDim.x); };
  f4 pre[2][NV];
  auto load_item = [&](f4 (&pr)[NV], int k) {
    const int b = k % NB, lo = R::new_lo(b);
    const int nv = (R::new_hi(b) - lo) * IW * 8;
    const f4* s4 = reinterpret_cast<const f4*>(X1 + ((int64_t)frame_of(k) * R::IH + lo) * IW * 32);
    // unconditional (clamped) loads: with loads under a branch the compiler cannot count
    // them and waits for vmcnt(0) — this band's and the next band's loads — at the split
#pragma unroll
    for (int j = 0; j < NV; ++j) pr[j] = s4[min(tid + j * 512, nv - 1)];
  };
  auto split_item = [&](const f4 (&pr)[NV], int k) {
    const int b = k % NB, lo = R::new_lo(b);
    const int nv = (R::new_hi(b) - lo) * IW * 8;
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      const int i = tid + j * 512;
      if (i < nv) {
        const int c4 = i & 7, px = i >> 3, y = lo + px / IW, x = px - (px / IW) * IW;
        uint2 t0, t1, t2;
        split3_pack(pr[j], t0, t1, t2);
        uint16_t* d = xs + (y % R::SLOTS) * RSP + ((x & 1) * WH + (x >> 1)) * PSX +
                      8 * ((c4 >> 1) ^ R::swz(y, x >> 1)) + 4 * (c4 & 1);
        *reinterpret_cast<uint2*>(d) = t0;
        *reinterpret_cast<uint2*>(d + PL) = t1;
        *reinterpret_cast<uint2*>(d + 2 * PL) = t2;
      }
    }
  };
  if (n_items > 0) {
    load_item(pre[0], 0);
    load_item(pre[1], min(1, n_items - 1));
    split_item(pre[0], 0);
    load_item(pre[0], min(2, n_items - 1));
  }
  __syncthreads();
  f4 acc[2];
  // band k's MFMAs, partial, split of k + 1 (pre[S1]) and loads of k + 3 into it
  auto band = [&](auto s1, int k) {
    constexpr int S1 = decltype(s1)::value;
    const int b = k % NB, oy0 = R::BR * b, nr = min(R::BR, R::OH - oy0);
#pragma unroll
    for (int u = 0; u < 2; ++u) acc[u] = f4zero();
    // tile t < 3: band row t, ox = i16; tile 3: row i16 >> 2, ox = 16 + (i16 & 3); a lane past the
    // band (or row 3 of tile 3) takes row 0 at its ox: the same pixel as another lane, so its
    // reads broadcast and its store repeats that lane's bytes
    const uint16_t* xb[2][2][2];  // [tile][ky - 2kh][kx >> 1]
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int t = tsel + 2 * u;
      int r = t < 3 ? t : (i16 >> 2), ox = t < 3 ? i16 : 16 + (i16 & 3);
      if (r >= nr) r = 0;
#pragma unroll
      for (int ky = 0; ky < 2; ++ky) {
        const int y = 2 * (oy0 + r) + 2 * kh + ky;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int xi = ox + h;
          xb[u][ky][h] = xs + (y % R::SLOTS) * RSP + xi * PSX + 8 * (q ^ R::swz(y, xi));
        }
      }
    }
    auto read_b = [&](bf16x8_t (&bv)[2][3], int i) {
      const int ky = i >> 2, kx = i & 3;
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const uint16_t* xp = xb[u][ky][kx >> 1] + (kx & 1) * WH * PSX;
#pragma unroll
        for (int tm = 0; tm < 3; ++tm) bv[u][tm] = *reinterpret_cast<const bf16x8_t*>(xp + tm * PL);
      }
    };
    auto mma = [&]() {
      bf16x8_t bv[2][2][3];  // [buffer][tile][term]: tap i + 1's fragments load under tap i's MFMAs
      read_b(bv[0], 0);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        if (i + 1 < 8) read_b(bv[(i + 1) & 1], i + 1);
#pragma unroll
        for (int u = 0; u < 2; ++u) {  // small terms first
          const bf16x8_t* bb = bv[i & 1][u];
          f4 c = acc[u];
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[i][2], bb[0], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[i][0], bb[2], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[i][1], bb[1], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[i][1], bb[0], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[i][0], bb[1], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[i][0], bb[0], c, 0, 0, 0);
          acc[u] = c;
        }
      }
      // lane (pixel i16, q) holds co ct*16 + 4q .. +3 of its pixel
      if (kh == 1) {
#pragma unroll
        for (int u = 0; u < 2; ++u)
          *reinterpret_cast<f4*>(part + ((k & 1) * TP + (tsel + 2 * u) * 16 + i16) * PP + ct * 16 + 4 * q) = acc[u];
      }
    };
    // next band's rows into the ring, then the loads of band k + 3 into the registers just
    // freed; past the last item both repeat the last one (same bytes into the same slots)
    auto stage = [&]() {
      split_item(pre[S1], min(k + 1, n_items - 1));
      load_item(pre[S1], min(k + 3, n_items - 1));
    };
    // the two waves of a SIMD (w and w + 4) take the phases in opposite orders, so one's split
    // (VALU, LDS writes) runs under the other's MFMAs instead of both idling the matrix pipe
    if (tsel == 0) {
      mma();
      stage();
    } else {
      stage();
      mma();
    }
  };
  auto epilogue = [&](int k) {
    if (kh != 0) return;
    const int b = k % NB, oy0 = R::BR * b, nr = min(R::BR, R::OH - oy0);
    const int64_t out0 = ((int64_t)frame_of(k) * NP + oy0 * OW) * 32 + ct * 16 + 4 * q;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int t = tsel + 2 * u;
      int r = t < 3 ? t : (i16 >> 2), ox = t < 3 ? i16 : 16 + (i16 & 3);
      if (r >= nr) r = 0;  // the pixel this lane computed (see band): same bytes as its own lane
      const f4 pv = *reinterpret_cast<const f4*>(part + ((k & 1) * TP + t * 16 + i16) * PP + ct * 16 + 4 * q);
      f4 v = acc[u] + pv;
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e] + b4[e], 0.0f);
      *reinterpret_cast<f4*>(X2 + out0 + (int64_t)(r * OW + ox) * 32) = v;
    }
  };
  for (int k = 0; k < n_items; k += 2) {
    band(std::integral_constant<int, 1>{}, k);
    __syncthreads();
    epilogue(k);
    if (k + 1 < n_items) {
      band(std::integral_constant<int, 0>{}, k + 1);
      __syncthreads();
      epilogue(k + 1);
    }
  }
}

// Two-workgroups-per-CU form of the ring kernel: the single 8-wave workgroup above keeps its
// MFMA pipe 47 % busy, bound by its per-band barrier and phase order rather than by HBM (a
// no-load ablation runs 10 % faster). Here a workgroup is 4 waves (role = (co tile, kernel-row
// half), each taking all 4 tiles of a band in two passes) over an 8-slot ring (74 KB of LDS):
// MFMA(b) -> partial -> barrier -> epilogue(b) + split of band b+1's rows over band b's six
// oldest slots + loads of band b+2 -> barrier. Its phases are serial, and the other workgroup
// on the CU fills them. Same sums in the same order as conv2_fwd_ring_kernel (bitwise).
struct Conv2Ring42x2 {
  static constexpr int SLOTS = 8, PL = SLOTS * Conv2Ring42::RSP;
  static constexpr int TP = 64, PP = 36;
  static constexpr int NV = (8 * Conv2Ring42::IW * 8 + 255) / 256;  // prefetched f4 per thread
  static constexpr size_t LDS = (size_t)3 * PL * 2 + (size_t)TP * PP * 4;
  static_assert(LDS <= 80 * 1024, "two workgroups per CU");
};

// PF (round 6): band k + 2's rows are loaded right after band k + 1's split and stay in flight
// through band k + 1's MFMAs (the PMC of the PF = false form: waves waiting 42 % of their
// cycles, most of it the split's wait on loads issued just before it); the split now precedes
// the epilogue, so its wait counts no X2 store. Same sums, same order: bitwise equal.
template <bool PF>
__global__ __launch_bounds__(256, 2) void conv2_fwd_ring2_kernel(const float* __restrict__ X1,
                                                                 const float* __restrict__ W2,
                                                                 const float* __restrict__ bias,
                                                                 float* __restrict__ X2, int n_frames, FrameList fl) {
  using R = Conv2Ring42;
  using Q = Conv2Ring42x2;
  constexpr int IW = R::IW, OW = R::OW, NB = R::NB, WH = R::WH, PSX = R::PSX, RSP = R::RSP, PL = Q::PL;
  constexpr int NV = Q::NV, PP = Q::PP, NP = R::OH * R::OW;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem_r3[];
  uint16_t* xs = reinterpret_cast<uint16_t*>(smem_r3);
  float* part = reinterpret_cast<float*>(smem_r3 + (size_t)3 * PL * 2);  // [TP][PP]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int ct = wave & 1, kh = wave >> 1;
  const int i16 = lane & 15, q = lane >> 4;
  bf16x8_t wf[8][3];  // [tap i: ky = 2kh + (i >> 2), kx = i & 3][term]: A[co = ct*16 + i16][k = ci 8q .. 8q+7]
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    union { uint16_t u[8]; bf16x8_t v; } t0, t1, t2;
    const float* wp = W2 + (ct * 16 + i16) * 512 + ((2 * kh + (i >> 2)) * 4 + (i & 3)) * 32 + 8 * q;
#pragma unroll
    for (int j = 0; j < 8; ++j) split3_bf16(wp[j], t0.u[j], t1.u[j], t2.u[j]);
    wf[i][0] = t0.v;
    wf[i][1] = t1.v;
    wf[i][2] = t2.v;
  }
  const f4 b4 = *reinterpret_cast<const f4*>(bias + ct * 16 + 4 * q);
  asm volatile("" ::"v"(b4[0]), "v"(b4[1]), "v"(b4[2]), "v"(b4[3]));  // landed before the loop
  n_frames = fl_count(fl, n_frames);
  const int my_frames = (int)blockIdx.x < n_frames ? (n_frames - 1 - (int)blockIdx.x) / (int)gridDim.x + 1 : 0;
  const int n_items = my_frames * NB;
  auto frame_of = [&](int k) { return fl_frame(fl, (int)blockIdx.x + (k / NB) * (int)gridDim.x); };
  // ring slot of X1 row y of item k's frame: rows of consecutive frames continue the count
  // (42 per frame), so a band's 8 rows and the next band's new rows (which replace the band's
  // six oldest once its MFMAs are done) never collide
  auto slot = [&](int k, int y) { return (42 * (k / NB) + y) & (Q::SLOTS - 1); };
  f4 pre[NV];
  auto load_item = [&](int k) {
    const int b = k % NB, lo = R::new_lo(b);
    const int nv = (R::new_hi(b) - lo) * IW * 8;
    const f4* s4 = reinterpret_cast<const f4*>(X1 + ((int64_t)frame_of(k) * R::IH + lo) * IW * 32);
#pragma unroll
    for (int j = 0; j < NV; ++j) pre[j] = s4[min(tid + j * 256, nv - 1)];
  };
  auto split_item = [&](int k) {
    const int b = k % NB, lo = R::new_lo(b);
    const int nv = (R::new_hi(b) - lo) * IW * 8;
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      const int i = tid + j * 256;
      if (i < nv) {
        const int c4 = i & 7, px = i >> 3, y = lo + px / IW, x = px - (px / IW) * IW;
        uint2 t0, t1, t2;
        split3_pack(pre[j], t0, t1, t2);
        uint16_t* d = xs + slot(k, y) * RSP + ((x & 1) * WH + (x >> 1)) * PSX +
                      8 * ((c4 >> 1) ^ R::swz(y, x >> 1)) + 4 * (c4 & 1);
        *reinterpret_cast<uint2*>(d) = t0;
        *reinterpret_cast<uint2*>(d + PL) = t1;
        *reinterpret_cast<uint2*>(d + 2 * PL) = t2;
      }
    }
  };
  if (n_items > 0) {
    load_item(0);
    split_item(0);
    if constexpr (PF) load_item(min(1, n_items - 1));
  }
  __syncthreads();
  f4 acc[4];
  for (int k = 0; k < n_items; ++k) {
    const int b = k % NB, oy0 = R::BR * b, nr = min(R::BR, R::OH - oy0);
    const int fk = frame_of(k);  // resolved here, where no LDS access is in flight
    // tile t < 3: band row t, ox = i16; tile 3: row i16 >> 2, ox = 16 + (i16 & 3); lanes past the
    // band take row 0 at their ox (see conv2_fwd_ring_kernel)
#pragma unroll
    for (int pass = 0; pass < 2; ++pass) {
      const uint16_t* xb[2][2][2];  // [tile][ky - 2kh][kx >> 1]
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int t = 2 * pass + u;
        int r = t < 3 ? t : (i16 >> 2);
        const int ox = t < 3 ? i16 : 16 + (i16 & 3);
        if (r >= nr) r = 0;
#pragma unroll
        for (int ky = 0; ky < 2; ++ky) {
          const int y = 2 * (oy0 + r) + 2 * kh + ky;
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int xi = ox + h;
            xb[u][ky][h] = xs + slot(k, y) * RSP + xi * PSX + 8 * (q ^ R::swz(y, xi));
          }
        }
      }
      auto read_b = [&](bf16x8_t (&bv)[2][3], int i) {
        const int ky = i >> 2, kx = i & 3;
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const uint16_t* xp = xb[u][ky][kx >> 1] + (kx & 1) * WH * PSX;
#pragma unroll
          for (int tm = 0; tm < 3; ++tm) bv[u][tm] = *reinterpret_cast<const bf16x8_t*>(xp + tm * PL);
        }
      };
      f4 c2[2] = {f4zero(), f4zero()};
      bf16x8_t bv[2][2][3];
      read_b(bv[0], 0);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        if (i + 1 < 8) read_b(bv[(i + 1) & 1], i + 1);
#pragma unroll
        for (int u = 0; u < 2; ++u) {  // small terms first
          const bf16x8_t* bb = bv[i & 1][u];
          f4 c = c2[u];
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[i][2], bb[0], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[i][0], bb[2], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[i][1], bb[1], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[i][1], bb[0], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[i][0], bb[1], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[i][0], bb[0], c, 0, 0, 0);
          c2[u] = c;
        }
      }
      acc[2 * pass] = c2[0];
      acc[2 * pass + 1] = c2[1];
    }
    if (kh == 1) {
#pragma unroll
      for (int t = 0; t < 4; ++t) *reinterpret_cast<f4*>(part + (t * 16 + i16) * PP + ct * 16 + 4 * q) = acc[t];
    }
    __syncthreads();  // MFMA(k) and the partials done: band k's oldest slots are free
    if constexpr (PF) {  // past the last item the split and the loads repeat it (same bytes, same slots)
      split_item(min(k + 1, n_items - 1));
      load_item(min(k + 2, n_items - 1));
    }
    if (kh == 0) {
      const int64_t out0 = ((int64_t)fk * NP + oy0 * OW) * 32 + ct * 16 + 4 * q;
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        int r = t < 3 ? t : (i16 >> 2);
        const int ox = t < 3 ? i16 : 16 + (i16 & 3);
        if (r >= nr) r = 0;
        const f4 pv = *reinterpret_cast<const f4*>(part + (t * 16 + i16) * PP + ct * 16 + 4 * q);
        f4 v = acc[t] + pv;
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e] + b4[e], 0.0f);
        *reinterpret_cast<f4*>(X2 + out0 + (int64_t)(r * OW + ox) * 32) = v;
      }
    }
    if constexpr (!PF) {
      if (k + 1 < n_items) {  // loaded here, not a band ahead: the other workgroup on the CU covers
        load_item(k + 1);     // the latency, and the 44 VGPRs keep the B fragments double-buffered
        split_item(k + 1);
      }
    }
    __syncthreads();  // band k + 1's rows in the ring, the partial buffer read
  }
}

// ---- conv1 + conv2 forward of a few envs at 174x174: one launch ------------------------------
// A rollout step of <= 16 envs (the logged run's 4) ran conv1_fwd_x3_kernel and then the banded
// conv2_fwd_x6_kernel, two dependent launches of ~10 us each, both bound by their load ->
// stage -> compute -> store chains rather than by their arithmetic. Here one workgroup takes one
// (frame, band of 3 conv2 output rows) item: it stages the image rows under the band's 8 X1
// rows (6 for the last band) as bf16, all 8 waves run conv1 on them (conv1_fwd_x3_kernel's
// product: split weight fragments in LDS, three accumulation chains, the same epilogue) into the
// ring kernel's split planes, and after one barrier the 8 waves run conv2 on the band with the
// ring kernel's roles and sums (conv2_fwd_ring_kernel: (co tile, kernel-row half, tile pair),
// the halves meeting through an LDS partial). The two X1 rows a band shares with the next are
// computed by both workgroups; X1 and the ReLU bitmask of a row go to HBM from one of them.
// X1 is bitwise conv1_fwd_x3_kernel's, X2 bitwise conv2_fwd_ring_kernel's.
struct Conv12Small174 {
  using R = Conv2Ring42;
  static constexpr int RB = 174 * 3, RS = (RB + 3) / 4 * 4;  // image row bytes / LDS row stride (bf16)
  static constexpr int ROWS = 8;                               // X1 rows of a band (6 for the last)
  static constexpr int IMG_ROWS = 4 * ROWS + 4;                // image rows under them (+ the ky = 7 pad row)
  static constexpr int ND = IMG_ROWS * RB / 4;                 // image dwords of a band
  static constexpr int NJ = (ND + 511) / 512;                  // image dwords per thread
  static constexpr int PLR = ROWS * R::RSP;                    // plane size (bf16)
  static constexpr size_t PLANES = (size_t)3 * PLR * 2, PART = (size_t)64 * 36 * 4;
  static constexpr size_t IMG = (size_t)IMG_ROWS * RS * 2, WFR = (size_t)kConv1X3WeightLds;
  static constexpr size_t LDS = PLANES + PART + IMG + WFR + 32 * 4;
  static_assert(LDS <= 160 * 1024, "conv12 small");
};

__global__ __launch_bounds__(512, 1) void conv12_small_kernel(FrameSrc src, int n_frames, const float* __restrict__ W1,
                                                              const float* __restrict__ b1,
                                                              const float* __restrict__ W2,
                                                              const float* __restrict__ b2, float* __restrict__ X1,
                                                              uint32_t* __restrict__ M1, float* __restrict__ X2) {
  using R = Conv2Ring42;
  using C = Conv12Small174;
  constexpr int IW = R::IW, OW = R::OW, NB = R::NB, WH = R::WH, PSX = R::PSX, RSP = R::RSP, PL = C::PLR;
  constexpr int NP = R::OH * R::OW, NPIX1 = R::IH * R::IW, RB = C::RB, RS = C::RS, NS = 11, PP = 36;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem_c12s[];
  uint16_t* xs = reinterpret_cast<uint16_t*>(smem_c12s);
  float* part = reinterpret_cast<float*>(smem_c12s + C::PLANES);                              // [64][PP]
  uint16_t* img = reinterpret_cast<uint16_t*>(smem_c12s + C::PLANES + C::PART);               // [IMG_ROWS][RS]
  bf16x8* bw = reinterpret_cast<bf16x8*>(smem_c12s + C::PLANES + C::PART + C::IMG);           // [NS][3][64]
  float* bsh = reinterpret_cast<float*>(smem_c12s + C::PLANES + C::PART + C::IMG + C::WFR);  // conv1 bias
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int it = blockIdx.x;  // grid = n_frames * NB (checked by the launcher)
  const int f = it / NB, b = it - (it / NB) * NB;
  const int y0 = 2 * R::BR * b, ny = min(C::ROWS, R::IH - y0);  // the band's X1 rows y0 .. y0 + ny - 1
  // image rows 4 y0 .. 4 (y0 + ny) + 3, issued first
  const int nd = (4 * ny + 4) * RB / 4;
  uint32_t pre[C::NJ];
  {
    const uint32_t* s4 = reinterpret_cast<const uint32_t*>(frame_ptr(src, f) + (int64_t)4 * y0 * RB);
#pragma unroll
    for (int j = 0; j < C::NJ; ++j) pre[j] = s4[min(tid + j * 512, nd - 1)];
  }
  // conv2's split weights for this wave's role, in registers (conv2_fwd_ring_kernel's)
  const int ct = wave & 1, kh = (wave >> 1) & 1, tsel = wave >> 2;
  const int i16 = lane & 15, q = lane >> 4;
  bf16x8_t wf[8][3];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    union { uint16_t u[8]; bf16x8_t v; } t0, t1, t2;
    const float* wp = W2 + (ct * 16 + i16) * 512 + ((2 * kh + (i >> 2)) * 4 + (i & 3)) * 32 + 8 * q;
#pragma unroll
    for (int j = 0; j < 8; ++j) split3_bf16(wp[j], t0.u[j], t1.u[j], t2.u[j]);
    wf[i][0] = t0.v;
    wf[i][1] = t1.v;
    wf[i][2] = t2.v;
  }
  const f4 b4 = *reinterpret_cast<const f4*>(b2 + ct * 16 + 4 * q);
  // conv1's split weight fragments [slice][term][lane] (conv1_fwd_x3_kernel's) and bias in LDS
  for (int i = tid; i < NS * 64; i += 512) {
    const int sl = i >> 6, ln = i & 63, hh = ln >> 5, co = ln & 31;
    union { uint16_t u[8]; bf16x8 v; } t0, t1, t2;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int kp = 16 * sl + 8 * hh + j, ky = kp / 24, kr = kp % 24;
      const float w = (ky < 7 && kr < 21) ? W1[co * 148 + ky * 21 + kr] : 0.0f;
      split3_bf16(w, t0.u[j], t1.u[j], t2.u[j]);
    }
    bw[(sl * 3 + 0) * 64 + ln] = t0.v;
    bw[(sl * 3 + 1) * 64 + ln] = t1.v;
    bw[(sl * 3 + 2) * 64 + ln] = t2.v;
  }
  if (tid < 32) bsh[tid] = b1[tid];
#pragma unroll
  for (int j = 0; j < C::NJ; ++j) {  // u8 -> bf16 rows (RB even: byte pairs never straddle a row)
    const int i = tid + j * 512;
    if (i < nd) stage_u8x4_bf16<RB, RS>(img, i, pre[j]);
  }
  __syncthreads();
  {  // conv1: tiles of 32 band pixels, wave w takes tiles w, w + 8
    const int h = lane >> 5, c32 = lane & 31, npx = ny * IW;
    const int tiles = (npx + 31) / 32;
    for (int t = wave; t < tiles; t += 8) {
      const int p = min(t * 32 + c32, npx - 1);
      const int yr = p / IW, x = p - (p / IW) * IW, y = y0 + yr;
      const uint16_t* base = img + (4 * yr) * RS + x * 12;
      int wl = lane;
      asm volatile("" : "+v"(wl));  // keeps the weight-fragment reads inside the tile loop
      f16v acc[3];
#pragma unroll
      for (int qq = 0; qq < 3; ++qq)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[qq][r] = 0.0f;
#pragma unroll
      for (int sl = 0; sl < NS; ++sl) {
        const int k0 = 16 * sl + 8 * h, ky = k0 / 24, kr0 = k0 - (k0 / 24) * 24;
        const uint2* qp = reinterpret_cast<const uint2*>(base + ky * RS + kr0);
        union { uint2 u[2]; bf16x8 v; } a;
        a.u[0] = qp[0];
        a.u[1] = qp[1];
#pragma unroll
        for (int qq = 0; qq < 3; ++qq)  // D^T = W^T A^T: rows = channels, columns = pixels
          acc[qq] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bw[(sl * 3 + qq) * 64 + wl], a.v, acc[qq], 0, 0, 0);
      }
      uint32_t bits = 0;
      f4 yv[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const f4 bj = *reinterpret_cast<const f4*>(bsh + 8 * j + 4 * h);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int i = 4 * j + r;
          const float sum = (acc[2][i] + acc[1][i]) + acc[0][i];
          yv[j][r] = fmaxf(sum * (1.0f / 255.0f) + bj[r], 0.0f);
          bits |= (yv[j][r] > 0.0f ? 1u : 0u) << (8 * j + 4 * h + r);
        }
      }
      bits |= (uint32_t)__shfl_xor((int)bits, 32);
      if (t * 32 + c32 < npx) {
        // X1 / bitmask rows y0 .. y0 + 5 from this band (all of the last band's)
        if (yr < 2 * R::BR || b == NB - 1) {
          const int64_t pix = (int64_t)f * NPIX1 + y * IW + x;
#pragma unroll
          for (int j = 0; j < 4; ++j) *reinterpret_cast<f4*>(X1 + pix * 32 + 8 * j + 4 * h) = yv[j];
          if (h == 0) M1[pix] = bits;
        }
        uint16_t* d = xs + yr * RSP + ((x & 1) * WH + (x >> 1)) * PSX + 4 * h;
        const int sw = R::swz(y, x >> 1);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          uint2 t0, t1, t2;
          split3_pack(yv[j], t0, t1, t2);
          uint16_t* dj = d + 8 * (j ^ sw);
          *reinterpret_cast<uint2*>(dj) = t0;
          *reinterpret_cast<uint2*>(dj + PL) = t1;
          *reinterpret_cast<uint2*>(dj + 2 * PL) = t2;
        }
      }
    }
  }
  __syncthreads();
  // conv2 on the band (conv2_fwd_ring_kernel's product and sums): plane row = y - y0
  const int oy0 = R::BR * b, nr = min(R::BR, R::OH - oy0);
  f4 acc[2] = {f4zero(), f4zero()};
  {
    const uint16_t* xb[2][2][2];  // [tile][ky - 2kh][kx >> 1]
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int t = tsel + 2 * u;
      int r = t < 3 ? t : (i16 >> 2);
      const int ox = t < 3 ? i16 : 16 + (i16 & 3);
      if (r >= nr) r = 0;
#pragma unroll
      for (int ky = 0; ky < 2; ++ky) {
        const int y = 2 * (oy0 + r) + 2 * kh + ky;
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {
          const int xi = ox + hh;
          xb[u][ky][hh] = xs + (y - y0) * RSP + xi * PSX + 8 * (q ^ R::swz(y, xi));
        }
      }
    }
    auto read_b = [&](bf16x8_t (&bv)[2][3], int i) {
      const int ky = i >> 2, kx = i & 3;
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const uint16_t* xp = xb[u][ky][kx >> 1] + (kx & 1) * WH * PSX;
#pragma unroll
        for (int tm = 0; tm < 3; ++tm) bv[u][tm] = *reinterpret_cast<const bf16x8_t*>(xp + tm * PL);
      }
    };
    bf16x8_t bv[2][2][3];
    read_b(bv[0], 0);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if (i + 1 < 8) read_b(bv[(i + 1) & 1], i + 1);
#pragma unroll
      for (int u = 0; u < 2; ++u) {  // small terms first (conv2_fwd_ring_kernel's order)
        const bf16x8_t* bb = bv[i & 1][u];
        f4 c = acc[u];
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[i][2], bb[0], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[i][0], bb[2], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[i][1], bb[1], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[i][1], bb[0], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[i][0], bb[1], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[i][0], bb[0], c, 0, 0, 0);
        acc[u] = c;
      }
    }
  }
  if (kh == 1) {
#pragma unroll
    for (int u = 0; u < 2; ++u)
      *reinterpret_cast<f4*>(part + ((tsel + 2 * u) * 16 + i16) * PP + ct * 16 + 4 * q) = acc[u];
  }
  __syncthreads();
  if (kh == 0) {
    const int64_t out0 = ((int64_t)f * NP + oy0 * OW) * 32 + ct * 16 + 4 * q;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int t = tsel + 2 * u;
      int r = t < 3 ? t : (i16 >> 2);
      const int ox = t < 3 ? i16 : 16 + (i16 & 3);
      if (r >= nr) r = 0;  // the pixel this lane computed: the same bytes as its own lane
      const f4 pv = *reinterpret_cast<const f4*>(part + (t * 16 + i16) * PP + ct * 16 + 4 * q);
      f4 v = acc[u] + pv;
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e] + b4[e], 0.0f);
      *reinterpret_cast<f4*>(X2 + out0 + (int64_t)(r * OW + ox) * 32) = v;
    }
  }
  (void)n_frames;
}

// Deterministic column sums of a [rows][32] matrix: per-block partials, then one block.
__global__ __launch_bounds__(256) void colsum32_partial_kernel(const float* __restrict__ A, int64_t rows,
                                                               float* __restrict__ partial) {
  const int c = threadIdx.x & 31, r0 = threadIdx.x >> 5;  // 8 row lanes per block
  float s = 0.0f;
  for (int64_t r = (int64_t)blockIdx.x * 8 + r0; r < rows; r += (int64_t)gridDim.x * 8) s += A[r * 32 + c];
  __shared__ float red[8][32];
  red[r0][c] = s;
  __syncthreads();
  if (threadIdx.x < 32) {
    float t = 0.0f;
    for (int i = 0; i < 8; ++i) t += red[i][threadIdx.x];
    partial[(int64_t)blockIdx.x * 32 + threadIdx.x] = t;
  }
}

__global__ void sum_slabs_kernel(const float* __restrict__ slab, int nslab, int64_t n, float* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float s = 0.0f;
  for (int z = 0; z < nslab; ++z) s += slab[(int64_t)z * n + i];
  out[i] = s;
}

}  // namespace vn
