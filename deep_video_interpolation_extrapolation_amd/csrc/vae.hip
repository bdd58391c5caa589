// vae.hip — the reparameterisation of VAEHRNet (reference nets/HRNet.py:960-966):
//   z = eps * exp(0.5 * logvar) + mu            (std = logvar.mul(0.5).exp_(); eps.mul(std).add_(mu))
// and its adjoint: gmu (+)= gz, glogvar (+)= gz * eps * 0.5 * exp(0.5 * logvar).
// eps is drawn by the caller (torch's device generator: std.new(std.size()).normal_()).
#include "common.h"

namespace dvie {

__global__ void reparam_fwd_kernel(const float* __restrict__ mu, const float* __restrict__ lv,
                                   const float* __restrict__ eps, float* __restrict__ z, long long n) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
    z[i] = eps[i] * expf(0.5f * lv[i]) + mu[i];
}

__global__ void reparam_bwd_kernel(const float* __restrict__ lv, const float* __restrict__ eps,
                                   const float* __restrict__ gz, float* __restrict__ gmu, float* __restrict__ glv,
                                   long long n, int beta) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const float g = gz[i];
    const float d = g * eps[i] * 0.5f * expf(0.5f * lv[i]);
    gmu[i] = beta ? gmu[i] + g : g;
    glv[i] = beta ? glv[i] + d : d;
  }
}

static int vae_grid(long long n) {
  long long b = (n + 255) / 256;
  return (int)(b < 1 ? 1 : (b > 4096 ? 4096 : b));
}

}  // namespace dvie

using namespace dvie;

extern "C" {

int dvie_reparam_fwd(const float* mu, const float* logvar, const float* eps, float* z, long long n, void* stream) {
  DVIE_CHECK_ARG(mu && logvar && eps && z && n >= 0, "reparam fwd: args");
  if (n == 0) return DVIE_OK;
  DVIE_LAUNCH(reparam_fwd_kernel, dim3(vae_grid(n)), dim3(256), 0, (hipStream_t)stream, mu, logvar, eps, z, n);
  DVIE_RETURN_LAUNCH();
}

int dvie_reparam_bwd(const float* logvar, const float* eps, const float* gz, float* gmu, float* glogvar, long long n,
                     int beta, void* stream) {
  DVIE_CHECK_ARG(logvar && eps && gz && gmu && glogvar && n >= 0, "reparam bwd: args");
  if (n == 0) return DVIE_OK;
  DVIE_LAUNCH(reparam_bwd_kernel, dim3(vae_grid(n)), dim3(256), 0, (hipStream_t)stream, logvar, eps, gz, gmu,
                     glogvar, n, beta);
  DVIE_RETURN_LAUNCH();
}

}  // extern "C"
