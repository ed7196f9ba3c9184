// Optimizer math shared by the W&D kernels (csrc/wide_deep.hip reductions + optimizers, csrc/wd_chain.hip's
// in-kernel tail): TF ApplyAdagrad / ApplyFtrl / Adam / SGD on one fp32 parameter (no epsilon in Adagrad, as TF),
// and the slab-column-order state (param / s0 / s1 indexed by gradient column; wsc[col]: -1 padding, -2 wide weight,
// >= 0 DNN weight with its bf16 weight-image offset). Included inside each translation unit's anonymous namespace.
#pragma once

struct OptHyper {
  int kind;        // 0 sgd, 1 adagrad, 2 ftrl, 3 adam
  float lr, beta1, beta2, eps, l1, l2, lr_power;
};

__device__ __forceinline__ float opt_update(const OptHyper& hp, float w, float g, float& a0, float& a1,
                                            long long step) {
  if (hp.kind == 0) return w - hp.lr * g;
  if (hp.kind == 1) {
    a0 += g * g;
    return w - hp.lr * g * rsqrtf(a0);
  }
  if (hp.kind == 2) {  // TF ApplyFtrl
    const float a = a0, an = a + g * g;
    float sq_new, sq_old;
    if (hp.lr_power == -0.5f) {
      sq_new = sqrtf(an);
      sq_old = sqrtf(a);
    } else {
      sq_new = powf(an, -hp.lr_power);
      sq_old = powf(a, -hp.lr_power);
    }
    a1 += g - (sq_new - sq_old) / hp.lr * w;
    const float quad = sq_new / hp.lr + 2.f * hp.l2;
    a0 = an;
    return fabsf(a1) > hp.l1 ? (copysignf(hp.l1, a1) - a1) / quad : 0.f;
  }
  a0 = hp.beta1 * a0 + (1.f - hp.beta1) * g;
  a1 = hp.beta2 * a1 + (1.f - hp.beta2) * g * g;
  const float bc1 = 1.f - powf(hp.beta1, (float)step);
  const float bc2 = 1.f - powf(hp.beta2, (float)step);
  return w - hp.lr * (a0 / bc1) / (sqrtf(a1 / bc2) + hp.eps);
}

// per-workgroup optimizer step slots (see csrc/wide_deep.hip)
constexpr int STEP_SLOTS = 512;

struct ScState {
  int w;           // wsc entry
  float p, a0, a1;
};
__device__ __forceinline__ ScState sc_load(int gi, int stride, const int* __restrict__ wsc, const float* __restrict__ param,
                                           const float* __restrict__ s0, const float* __restrict__ s1) {
  ScState st{-1, 0.f, 0.f, 0.f};
  if (gi < stride) {
    st.w = wsc[gi];
    st.p = param[gi];
    st.a0 = s0[gi];
    st.a1 = s1[gi];
  }
  return st;
}
__device__ __forceinline__ void sc_update(int gi, ScState st, float g, const OptHyper& hd, const OptHyper& hw,
                                          long long step, float* __restrict__ param, float* __restrict__ s0,
                                          float* __restrict__ s1, uint16_t* __restrict__ wt_out) {
  if (st.w == -1) return;
  const float w = opt_update(st.w >= 0 ? hd : hw, st.p, g, st.a0, st.a1, step);
  s0[gi] = st.a0;
  s1[gi] = st.a1;
  param[gi] = w;
  if (st.w >= 0) wt_out[st.w] = __builtin_bit_cast(uint16_t, (bf16)w);
}

