// Window-hash kernels: XCodecHash (xcodec/xcodec_hash.h:31-177) at every
// offset, and per whole segment (tack -h, programs/tack/tack.cc:368-414).
//
// One wave per 2048 window positions.  Lane l owns the 32 consecutive
// positions [p + 32 l, p + 32 l + 32); its first window's sums come from two
// wave prefix scans over per-lane 32-byte segment sums (segments [l, l+64) of
// the 4 KiB span [p, p + 4096)), then the lane rolls exactly like
// RollingHash::roll (xcodec_hash.h:57-70).
#include "xcg_device.h"

namespace xcg {

__global__ __launch_bounds__(256) void window_hashes_kernel(const uint8_t* __restrict__ x, int64_t len,
                                                            uint64_t* __restrict__ out) {
  const int64_t npos = len - SEG + 1;
  const int64_t wave = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t p = wave * SEG;
  if (p >= npos) return;
  const int l = lane_id();
  const int64_t q0 = p + 32 * l;
  u32x4 a0 = load16_guarded(x, q0, len), a1 = load16_guarded(x, q0 + 16, len);
  u32x4 b0 = load16_guarded(x, q0 + SEG, len), b1 = load16_guarded(x, q0 + SEG + 16, len);
  const uint32_t xa[8] = {a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]};
  const uint32_t xb[8] = {b0[0], b0[1], b0[2], b0[3], b1[0], b1[1], b1[2], b1[3]};
  uint32_t sxa = 0, sqxa = 0, sfa = 0, sqfa = 0, sxb = 0, sqxb = 0, sfb = 0, sqfb = 0;
#pragma unroll
  for (int j = 0; j < 32; ++j) {
    const uint32_t va = byte_of(xa[j >> 2], j & 3), vb = byte_of(xb[j >> 2], j & 3);
    const uint32_t fa = ffbl(va) + 1u, fb = ffbl(vb) + 1u;
    sxa += va; sqxa += j * va; sfa += fa; sqfa += j * fa;
    sxb += vb; sqxb += j * vb; sfb += fb; sqfb += j * fb;
  }
  const uint32_t qa = 32u * l, qb = 2048u + 32u * l;
  const uint32_t ta = qa * sxa + sqxa, tb = qb * sxb + sqxb;
  const uint32_t tfa = qa * sfa + sqfa, tfb = qb * sfb + sqfb;
  const uint32_t dx = sxb - sxa, dt = tb - ta, df = sfb - sfa, dtf = tfb - tfa;
  uint32_t X1 = wave_sum(sxa) + wave_incl_scan(dx) - dx;
  const uint32_t TT = wave_sum(ta) + wave_incl_scan(dt) - dt;
  uint32_t F1 = wave_sum(sfa) + wave_incl_scan(df) - df;
  const uint32_t TF = wave_sum(tfa) + wave_incl_scan(dtf) - dtf;
  uint32_t X2c = (2048u + qa) * X1 - TT + CLO;
  uint32_t F2 = (2048u + qa) * F1 - TF;
#pragma unroll
  for (int j = 0; j < 32; ++j) {
    const int64_t s = q0 + j;
    if (s < npos) {
      const uint32_t lo = (X1 << 20) + X2c;
      const uint32_t hi = ((F1 << 16) + F2) << 4;
      out[s] = ((uint64_t)hi << 32) | lo;
    }
    const uint32_t xo = byte_of(xa[j >> 2], j & 3), xn = byte_of(xb[j >> 2], j & 3);
    const uint32_t ro = ffbl(xo), rn = ffbl(xn);
    X1 = X1 + xn - xo;
    X2c = X2c + X1 - (xo << 11);
    F1 = F1 + rn - ro;
    F2 = F2 + F1 - (ro << 11) - 2048u;
  }
}

// One thread per 2048-byte segment: XCodecHash::hash (add() x 2048), stored
// big-endian like tack -h's BigEndian::encode (programs/tack/tack.cc:388-390).
__global__ __launch_bounds__(256) void segment_hashes_kernel(const uint8_t* __restrict__ x, int64_t nseg,
                                                             uint64_t* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nseg) return;
  const u32x4* w = (const u32x4*)(x + i * SEG);   // 16-byte aligned if x is
  uint32_t X1 = 0, X2 = 0, F1 = 0, F2 = 0;
  for (int k = 0; k < SEG / 16; ++k) {
    const u32x4 v = *(const u32x4_u*)(w + k);
#pragma unroll
    for (int b = 0; b < 16; ++b) {
      const uint32_t c = byte_of(v[b >> 2], b & 3);
      const uint32_t f = ffbl(c) + 1u;
      const uint32_t wt = 2048u - (16u * k + b);
      X1 += c; X2 += wt * c; F1 += f; F2 += wt * f;
    }
  }
  const uint32_t lo = (X1 << 20) + X2 + CLO;
  const uint32_t hi = ((F1 << 16) + F2) << 4;
  out[i] = __builtin_bswap64(((uint64_t)hi << 32) | lo);
}

}  // namespace xcg

extern "C" int xcg_launch_window_hashes(const uint8_t* d_x, uint64_t len, uint64_t* d_hash, hipStream_t stream) {
  if (len < (uint64_t)xcg::SEG) return 0;
  const uint64_t npos = len - xcg::SEG + 1;
  const uint64_t waves = (npos + xcg::SEG - 1) / xcg::SEG;
  hipLaunchKernelGGL(xcg::window_hashes_kernel, dim3((unsigned)((waves + 3) / 4)), dim3(256), 0, stream, d_x,
                     (int64_t)len, d_hash);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

extern "C" int xcg_launch_segment_hashes(const uint8_t* d_x, uint64_t len, uint64_t* d_hash, hipStream_t stream) {
  const uint64_t nseg = len / xcg::SEG;
  if (nseg == 0) return 0;
  hipLaunchKernelGGL(xcg::segment_hashes_kernel, dim3((unsigned)((nseg + 255) / 256)), dim3(256), 0, stream, d_x,
                     (int64_t)nseg, d_hash);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}
