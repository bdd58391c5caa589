// Cityscapes clip preparation on the device: flip + crop + to_tensor/normalize of the RGB
// frames and the 20-class one-hot of the label maps, read straight from an HBM-resident
// uint8 clip store.  Reference: folder.py:211-247 (train), 248-261 (val).
//
// HBM-bound byte work (4 B read, 12 + 4*n_classes B written per output pixel): a thread
// owns 4 consecutive output pixels of a row, so every plane store is a 16-byte vector and a
// wave writes 1 KiB contiguous runs per plane.  No MFMA, no LDS.
#include "common.h"

namespace dvie {

template <bool kV4>
__global__ __launch_bounds__(256) void clip_prep_kernel(const dvie_clip_desc p) {
  const int wq = (p.wc + 3) >> 2;
  const long long hwc = (long long)p.hc * p.wc;
  const long long total = (long long)p.b * p.t * p.hc * wq;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < total;
       e += (long long)gridDim.x * blockDim.x) {
    const int xq = (int)(e % wq);
    long long r = e / wq;
    const int y = (int)(r % p.hc);
    r /= p.hc;
    const int t = (int)(r % p.t), b = (int)(r / p.t);
    const int* pr = p.params + ((long long)b * p.t + t) * 3;
    const int flip = pr[0], h1 = pr[1], w1 = pr[2];
    const long long clip = p.idx ? p.idx[b] : b;
    const long long frame = clip * p.t + t;
    const uint8_t* row = p.img + (frame * p.h0 + (h1 + y)) * (long long)p.w0 * 3;
    const uint8_t* srow = p.seg ? p.seg + (frame * p.h0 + (h1 + y)) * (long long)p.w0 : nullptr;
    float rgb[3][4];
    int lab[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int x = 4 * xq + k;
      const int xs = x < p.wc ? (flip ? p.w0 - 1 - (w1 + x) : w1 + x) : 0;
#pragma unroll
      for (int c = 0; c < 3; ++c) rgb[c][k] = ((float)row[xs * 3 + c] / 255.f - 0.5f) / 0.5f;
      lab[k] = srow ? (int)srow[xs] : 0;
    }
    const long long o = (long long)y * p.wc + 4 * xq;
    float* fr = p.frames + ((long long)t * p.b + b) * 3 * hwc;
    if (kV4) {
#pragma unroll
      for (int c = 0; c < 3; ++c) *(f32x4*)(fr + c * hwc + o) = f32x4{rgb[c][0], rgb[c][1], rgb[c][2], rgb[c][3]};
    } else {
      for (int k = 0; k < 4 && 4 * xq + k < p.wc; ++k)
        for (int c = 0; c < 3; ++c) fr[c * hwc + o + k] = rgb[c][k];
    }
    if (srow) {
      float* sg = p.segs + ((long long)t * p.b + b) * p.n_classes * hwc;
      for (int cls = 0; cls < p.n_classes; ++cls) {
        if (kV4) {
          *(f32x4*)(sg + cls * hwc + o) = f32x4{lab[0] == cls ? 1.f : 0.f, lab[1] == cls ? 1.f : 0.f,
                                                lab[2] == cls ? 1.f : 0.f, lab[3] == cls ? 1.f : 0.f};
        } else {
          for (int k = 0; k < 4 && 4 * xq + k < p.wc; ++k) sg[cls * hwc + o + k] = lab[k] == cls ? 1.f : 0.f;
        }
      }
      if (p.bad) {
        int nb = 0;
        for (int k = 0; k < 4; ++k) nb += (4 * xq + k < p.wc && lab[k] >= p.n_classes) ? 1 : 0;
        if (nb) atomicAdd(p.bad, nb);
      }
    }
  }
}

}  // namespace dvie

using namespace dvie;

extern "C" {

int dvie_clip_prep(const dvie_clip_desc* d, void* stream) {
  DVIE_CHECK_ARG(d && d->img && d->params && d->frames && d->b > 0 && d->t > 0 && d->hc > 0 && d->wc > 0 &&
                     d->hc <= d->h0 && d->wc <= d->w0,
                 "clip_prep: args");
  DVIE_CHECK_ARG(!d->seg || (d->segs && d->n_classes > 0 && d->n_classes <= 255), "clip_prep: seg args");
  const bool v4 = d->wc % 4 == 0 && ((uintptr_t)d->frames & 15) == 0 && (!d->seg || ((uintptr_t)d->segs & 15) == 0);
  const long long total = (long long)d->b * d->t * d->hc * ((d->wc + 3) / 4);
  long long blocks = (total + 255) / 256;
  if (blocks > 16384) blocks = 16384;
  if (v4)
    DVIE_LAUNCH(clip_prep_kernel<true>, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, *d);
  else
    DVIE_LAUNCH(clip_prep_kernel<false>, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, *d);
  DVIE_RETURN_LAUNCH();
}

}  // extern "C"
