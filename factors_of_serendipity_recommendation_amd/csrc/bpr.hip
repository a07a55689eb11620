// the BPR minibatch loss and its gradient as two fused kernels.
//
// Reference: LightGCN.bpr_loss (lightGCN/LightGCN-PyTorch-master/code/model.py:196-209) over
// getEmbedding (model.py:186-194), driven by utils.BPRLoss.stageOne (code/utils.py:43-52):
//   loss = mean_b softplus(<u_b, n_b> - <u_b, p_b>)          (light rows: the propagated table)
//   reg  = 0.5 * (|U0|^2 + |P0|^2 + |N0|^2) / B               (ego rows: the embedding weights)
// In torch that is ~12 forward kernels and, in backward, three index_put/embedding backward
// scatters (each a sort) plus the elementwise chain.  Here:
//   forward : one 16-lane group per triple reads its 6 rows once, writes sigmoid(x) per triple and
//             one (loss, reg) partial per workgroup; a one-workgroup pass sums the partials in a
//             fixed order (deterministic, no atomics).
//   backward: one group per triple scales the same rows by the upstream gradients (read from device
//             memory, no host sync) and adds them into the dense gradients with f32 atomics --
//             the same non-deterministic summation order torch's index_put_(accumulate) has.
// A triple with an index out of range poisons the loss with NaN instead of faulting.
#include "lgx_common.h"

#include <algorithm>
#include <cmath>

namespace lgx {
namespace {

constexpr int kGroup = 16;          // lanes per triple: a d=64 f32 row is 16 x float4
constexpr int kThreads = 256;       // 16 triples per workgroup

__device__ __forceinline__ float group_sum(float v) {
#pragma unroll
    for (int o = kGroup / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, kGroup);
    return v;
}

// torch.nn.functional.softplus(x), beta 1, threshold 20
__device__ __forceinline__ float softplus(float x) { return x > 20.f ? x : log1pf(expf(x)); }

struct Rows {
    const float* u;
    const float* p;
    const float* n;
    const float* eu;
    const float* ep;
    const float* en;
};

__device__ __forceinline__ bool triple_rows(const float* light, const float* ego_user, const float* ego_item,
                                            int64_t n_users, int64_t n_items, int64_t d, int64_t u, int64_t p,
                                            int64_t n, Rows& r) {
    if (u < 0 || u >= n_users || p < 0 || p >= n_items || n < 0 || n >= n_items) return false;
    r.u = light + u * d;
    r.p = light + (n_users + p) * d;
    r.n = light + (n_users + n) * d;
    r.eu = ego_user + u * d;
    r.ep = ego_item + p * d;
    r.en = ego_item + n * d;
    return true;
}

template <bool VEC>
__global__ __launch_bounds__(kThreads) void bpr_forward_kernel(const float* __restrict__ light,
                                                              const float* __restrict__ ego_user,
                                                              const float* __restrict__ ego_item, int64_t n_users,
                                                              int64_t n_items, int64_t d,
                                                              const int64_t* __restrict__ users,
                                                              const int64_t* __restrict__ pos,
                                                              const int64_t* __restrict__ neg, int64_t B,
                                                              float* __restrict__ coef, float2* __restrict__ partials) {
    __shared__ float2 red[kThreads / kGroup];
    const int lane = threadIdx.x % kGroup, g = threadIdx.x / kGroup;
    const int64_t b = blockIdx.x * (int64_t)(kThreads / kGroup) + g;
    float loss = 0.f, reg = 0.f;
    if (b < B) {
        Rows r;
        float sp = 0.f, sn = 0.f;
        if (triple_rows(light, ego_user, ego_item, n_users, n_items, d, users[b], pos[b], neg[b], r)) {
            if (VEC) {
                for (int64_t j = lane * 4; j < d; j += kGroup * 4) {
                    const float4 u = *reinterpret_cast<const float4*>(r.u + j);
                    const float4 p = *reinterpret_cast<const float4*>(r.p + j);
                    const float4 n = *reinterpret_cast<const float4*>(r.n + j);
                    const float4 a = *reinterpret_cast<const float4*>(r.eu + j);
                    const float4 c = *reinterpret_cast<const float4*>(r.ep + j);
                    const float4 e = *reinterpret_cast<const float4*>(r.en + j);
                    sp += u.x * p.x + u.y * p.y + u.z * p.z + u.w * p.w;
                    sn += u.x * n.x + u.y * n.y + u.z * n.z + u.w * n.w;
                    reg += a.x * a.x + a.y * a.y + a.z * a.z + a.w * a.w + c.x * c.x + c.y * c.y + c.z * c.z +
                           c.w * c.w + e.x * e.x + e.y * e.y + e.z * e.z + e.w * e.w;
                }
            } else {
                for (int64_t j = lane; j < d; j += kGroup) {
                    sp += r.u[j] * r.p[j];
                    sn += r.u[j] * r.n[j];
                    reg += r.eu[j] * r.eu[j] + r.ep[j] * r.ep[j] + r.en[j] * r.en[j];
                }
            }
            sp = group_sum(sp);
            sn = group_sum(sn);
            reg = group_sum(reg);
            const float x = sn - sp;
            loss = softplus(x);
            if (lane == 0) coef[b] = 1.f / (1.f + expf(-x));  // d softplus / dx
        } else {
            loss = __builtin_nanf("");
            if (lane == 0) coef[b] = 0.f;
        }
    }
    if (lane == 0) red[g] = make_float2(loss, reg);
    __syncthreads();
    if (threadIdx.x == 0) {
        float2 s = make_float2(0.f, 0.f);
        for (int i = 0; i < kThreads / kGroup; ++i) {
            s.x += red[i].x;
            s.y += red[i].y;
        }
        partials[blockIdx.x] = s;
    }
}

// loss = sum(softplus) / B (torch.mean), reg = 0.5 * sum(sq) / B; partials summed in a fixed order
__global__ __launch_bounds__(kThreads) void bpr_finalize_kernel(const float2* __restrict__ partials, int64_t n_part,
                                                               int64_t B, float* __restrict__ out_loss,
                                                               float* __restrict__ out_reg) {
    __shared__ float2 red[kThreads];
    float2 s = make_float2(0.f, 0.f);
    for (int64_t i = threadIdx.x; i < n_part; i += kThreads) {
        s.x += partials[i].x;
        s.y += partials[i].y;
    }
    red[threadIdx.x] = s;
    __syncthreads();
    for (int o = kThreads / 2; o > 0; o >>= 1) {
        if (threadIdx.x < o) {
            red[threadIdx.x].x += red[threadIdx.x + o].x;
            red[threadIdx.x].y += red[threadIdx.x + o].y;
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        *out_loss = red[0].x / (float)B;
        *out_reg = 0.5f * red[0].y / (float)B;
    }
}

template <bool VEC>
__global__ __launch_bounds__(kThreads) void bpr_backward_kernel(const float* __restrict__ light,
                                                               const float* __restrict__ ego_user,
                                                               const float* __restrict__ ego_item, int64_t n_users,
                                                               int64_t n_items, int64_t d,
                                                               const int64_t* __restrict__ users,
                                                               const int64_t* __restrict__ pos,
                                                               const int64_t* __restrict__ neg, int64_t B,
                                                               const float* __restrict__ coef,
                                                               const float* __restrict__ grad_loss,
                                                               const float* __restrict__ grad_reg,
                                                               float* __restrict__ g_light, float* __restrict__ g_user,
                                                               float* __restrict__ g_item) {
    const int lane = threadIdx.x % kGroup, g = threadIdx.x / kGroup;
    const int64_t b = blockIdx.x * (int64_t)(kThreads / kGroup) + g;
    if (b >= B) return;
    const int64_t u = users[b], p = pos[b], n = neg[b];
    Rows r;
    if (!triple_rows(light, ego_user, ego_item, n_users, n_items, d, u, p, n, r)) return;
    const float c = *grad_loss * coef[b] / (float)B;  // d loss / d x_b
    const float s = *grad_reg / (float)B;             // d reg / d ego row = s * row
    float* gu = g_light + u * d;
    float* gp = g_light + (n_users + p) * d;
    float* gn = g_light + (n_users + n) * d;
    float* geu = g_user + u * d;
    float* gep = g_item + p * d;
    float* gen = g_item + n * d;
    auto one = [&](int64_t j) {
        const float uu = r.u[j], pp = r.p[j], nn = r.n[j];
        unsafeAtomicAdd(gu + j, c * (nn - pp));  // x = <u,n> - <u,p>
        unsafeAtomicAdd(gp + j, -c * uu);
        unsafeAtomicAdd(gn + j, c * uu);
        unsafeAtomicAdd(geu + j, s * r.eu[j]);
        unsafeAtomicAdd(gep + j, s * r.ep[j]);
        unsafeAtomicAdd(gen + j, s * r.en[j]);
    };
    if (VEC) {
        for (int64_t j = lane * 4; j < d; j += kGroup * 4) {
            one(j);
            one(j + 1);
            one(j + 2);
            one(j + 3);
        }
    } else {
        for (int64_t j = lane; j < d; j += kGroup) one(j);
    }
}

}  // namespace
}  // namespace lgx

using namespace lgx;

extern "C" int lgx_bpr_loss_workspace(int64_t B, size_t* ws_bytes) {
    LGX_REQUIRE(B >= 0 && ws_bytes, LGX_ERR_INVALID_ARG, "lgx_bpr_loss_workspace: bad arguments");
    *ws_bytes = align_up((size_t)std::max<int64_t>(1, ceil_div(B, kThreads / kGroup)) * sizeof(float2));
    return LGX_OK;
}

extern "C" int lgx_bpr_loss_forward(const float* light, const float* ego_user, const float* ego_item, int64_t n_users,
                                    int64_t n_items, int64_t d, const int64_t* users, const int64_t* pos,
                                    const int64_t* neg, int64_t B, float* coef, float* out_loss, float* out_reg, void* ws,
                                    size_t ws_bytes, lgx_stream_t stream) {
    LGX_REQUIRE(n_users > 0 && n_items > 0 && d > 0 && B > 0, LGX_ERR_INVALID_ARG, "lgx_bpr_loss_forward: bad sizes");
    LGX_REQUIRE(light && ego_user && ego_item && users && pos && neg && coef && out_loss && out_reg && ws, LGX_ERR_INVALID_ARG,
                "lgx_bpr_loss_forward: null pointer");
    const int64_t nblk = ceil_div(B, kThreads / kGroup);
    size_t need = 0;
    lgx_bpr_loss_workspace(B, &need);
    LGX_REQUIRE(ws_bytes >= need, LGX_ERR_WORKSPACE, "lgx_bpr_loss_forward: workspace %zu < %zu", ws_bytes, need);
    const bool vec = d % 4 == 0 && ((uintptr_t)light | (uintptr_t)ego_user | (uintptr_t)ego_item) % 16 == 0;
    float2* part = static_cast<float2*>(ws);
    if (vec)
        bpr_forward_kernel<true><<<(unsigned)nblk, kThreads, 0, as_hip(stream)>>>(
            light, ego_user, ego_item, n_users, n_items, d, users, pos, neg, B, coef, part);
    else
        bpr_forward_kernel<false><<<(unsigned)nblk, kThreads, 0, as_hip(stream)>>>(
            light, ego_user, ego_item, n_users, n_items, d, users, pos, neg, B, coef, part);
    LGX_LAUNCH_CHECK();
    bpr_finalize_kernel<<<1, kThreads, 0, as_hip(stream)>>>(part, nblk, B, out_loss, out_reg);
    LGX_LAUNCH_CHECK();
    return LGX_OK;
}

extern "C" int lgx_bpr_loss_backward(const float* light, const float* ego_user, const float* ego_item,
                                     int64_t n_users, int64_t n_items, int64_t d, const int64_t* users,
                                     const int64_t* pos, const int64_t* neg, int64_t B, const float* coef,
                                     const float* grad_loss, const float* grad_reg, float* g_light, float* g_user, float* g_item,
                                     lgx_stream_t stream) {
    LGX_REQUIRE(n_users > 0 && n_items > 0 && d > 0 && B > 0, LGX_ERR_INVALID_ARG, "lgx_bpr_loss_backward: bad sizes");
    LGX_REQUIRE(light && ego_user && ego_item && users && pos && neg && coef && grad_loss && grad_reg && g_light && g_user && g_item,
                LGX_ERR_INVALID_ARG, "lgx_bpr_loss_backward: null pointer");
    const int64_t nblk = ceil_div(B, kThreads / kGroup);
    const bool vec = d % 4 == 0 && ((uintptr_t)light | (uintptr_t)ego_user | (uintptr_t)ego_item) % 16 == 0;
    if (vec)
        bpr_backward_kernel<true><<<(unsigned)nblk, kThreads, 0, as_hip(stream)>>>(
            light, ego_user, ego_item, n_users, n_items, d, users, pos, neg, B, coef, grad_loss, grad_reg, g_light, g_user,
            g_item);
    else
        bpr_backward_kernel<false><<<(unsigned)nblk, kThreads, 0, as_hip(stream)>>>(
            light, ego_user, ego_item, n_users, n_items, d, users, pos, neg, B, coef, grad_loss, grad_reg, g_light, g_user,
            g_item);
    LGX_LAUNCH_CHECK();
    return LGX_OK;
}

// ------------------------------------------------------------------------------ Adam step
// utils.BPRLoss's optimizer is torch.optim.Adam (code/utils.py:36-41; no weight decay, no amsgrad).
// torch runs it as ~7 multi-tensor passes over (param, grad, exp_avg, exp_avg_sq); this is one
// pass: 16 B read + 12 B written per parameter, float4 per lane.  Same update as torch's:
//   m = lerp(m, g, 1 - beta1); v = beta2 v + (1 - beta2) g^2;
//   p -= step_size * m / (sqrt(v) / bc2_sqrt + eps)   with step_size = lr / (1 - beta1^t).
namespace lgx {
namespace {

struct AdamArgs {
    float w1, beta2, w2, step_size, bc2_sqrt, eps;
};

__device__ __forceinline__ void adam_one(float& p, float g, float& m, float& v, const AdamArgs& a) {
    const float diff = g - m;  // torch lerp: weight < 0.5 ? self + w * diff : end - diff * (1 - w)
    m = a.w1 < 0.5f ? m + a.w1 * diff : g - diff * (1.f - a.w1);
    v = v * a.beta2 + a.w2 * g * g;
    p = p - a.step_size * (m / (sqrtf(v) / a.bc2_sqrt + a.eps));
}

__global__ __launch_bounds__(256) void adam_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                  float* __restrict__ m, float* __restrict__ v, int64_t n,
                                                  AdamArgs a) {
    const int64_t i4 = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    const int64_t i = i4 * 4;
    if (i + 3 < n) {
        float4 P = reinterpret_cast<float4*>(p)[i4];
        const float4 G = reinterpret_cast<const float4*>(g)[i4];
        float4 M = reinterpret_cast<float4*>(m)[i4];
        float4 V = reinterpret_cast<float4*>(v)[i4];
        adam_one(P.x, G.x, M.x, V.x, a);
        adam_one(P.y, G.y, M.y, V.y, a);
        adam_one(P.z, G.z, M.z, V.z, a);
        adam_one(P.w, G.w, M.w, V.w, a);
        reinterpret_cast<float4*>(p)[i4] = P;
        reinterpret_cast<float4*>(m)[i4] = M;
        reinterpret_cast<float4*>(v)[i4] = V;
    } else {
        for (int64_t j = i; j < n; ++j) adam_one(p[j], g[j], m[j], v[j], a);
    }
}

// the same step with t read from device memory (a graph-captured training step replays with the
// counter the captured add advanced): the bias corrections in double per thread, rounded once
struct AdamDevArgs {
    float w1, beta2, w2, eps;
    double lr, b1, b2;
};
__global__ __launch_bounds__(256) void adam_kernel_dev(float* __restrict__ p, const float* __restrict__ g,
                                                      float* __restrict__ m, float* __restrict__ v, int64_t n,
                                                      AdamDevArgs h, const float* __restrict__ step) {
    const double t = (double)*step;
    const AdamArgs a{h.w1, h.beta2, h.w2, (float)(h.lr / (1.0 - pow(h.b1, t))), (float)sqrt(1.0 - pow(h.b2, t)),
                     h.eps};
    const int64_t i4 = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    const int64_t i = i4 * 4;
    if (i + 3 < n) {
        float4 P = reinterpret_cast<float4*>(p)[i4];
        const float4 G = reinterpret_cast<const float4*>(g)[i4];
        float4 M = reinterpret_cast<float4*>(m)[i4];
        float4 V = reinterpret_cast<float4*>(v)[i4];
        adam_one(P.x, G.x, M.x, V.x, a);
        adam_one(P.y, G.y, M.y, V.y, a);
        adam_one(P.z, G.z, M.z, V.z, a);
        adam_one(P.w, G.w, M.w, V.w, a);
        reinterpret_cast<float4*>(p)[i4] = P;
        reinterpret_cast<float4*>(m)[i4] = M;
        reinterpret_cast<float4*>(v)[i4] = V;
    } else {
        for (int64_t j = i; j < n; ++j) adam_one(p[j], g[j], m[j], v[j], a);
    }
}

}  // namespace
}  // namespace lgx

extern "C" int lgx_adam_step_dev(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, int64_t n,
                                 double lr, double beta1, double beta2, double eps, const float* step,
                                 lgx_stream_t stream) {
    LGX_REQUIRE(n >= 0 && lr >= 0.0 && beta1 >= 0.0 && beta1 < 1.0 && beta2 >= 0.0 && beta2 < 1.0, LGX_ERR_INVALID_ARG,
                "lgx_adam_step_dev: bad arguments");
    if (n == 0) return LGX_OK;
    LGX_REQUIRE(param && grad && exp_avg && exp_avg_sq && step, LGX_ERR_INVALID_ARG, "lgx_adam_step_dev: null pointer");
    LGX_REQUIRE(((uintptr_t)param | (uintptr_t)grad | (uintptr_t)exp_avg | (uintptr_t)exp_avg_sq) % 16 == 0,
                LGX_ERR_INVALID_ARG, "lgx_adam_step_dev: tensors must be 16-byte aligned");
    AdamDevArgs h{(float)(1.0 - beta1), (float)beta2, (float)(1.0 - beta2), (float)eps, lr, beta1, beta2};
    const int64_t n4 = ceil_div(n, (int64_t)4);
    adam_kernel_dev<<<(unsigned)ceil_div(n4, (int64_t)256), 256, 0, as_hip(stream)>>>(param, grad, exp_avg, exp_avg_sq,
                                                                                      n, h, step);
    LGX_LAUNCH_CHECK();
    return LGX_OK;
}

extern "C" int lgx_adam_step(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, int64_t n, double lr,
                             double beta1, double beta2, double eps, int64_t step, lgx_stream_t stream) {
    LGX_REQUIRE(n >= 0 && step >= 1 && lr >= 0.0 && beta1 >= 0.0 && beta1 < 1.0 && beta2 >= 0.0 && beta2 < 1.0,
                LGX_ERR_INVALID_ARG, "lgx_adam_step: bad arguments");
    if (n == 0) return LGX_OK;
    LGX_REQUIRE(param && grad && exp_avg && exp_avg_sq, LGX_ERR_INVALID_ARG, "lgx_adam_step: null pointer");
    LGX_REQUIRE(((uintptr_t)param | (uintptr_t)grad | (uintptr_t)exp_avg | (uintptr_t)exp_avg_sq) % 16 == 0,
                LGX_ERR_INVALID_ARG, "lgx_adam_step: tensors must be 16-byte aligned");
    // every scalar in double on the host and rounded once to f32, as torch's Adam derives them from
    // Python floats (1 - beta2 in f32 arithmetic would be 1.3e-5 off)
    const double bc1 = 1.0 - std::pow(beta1, (double)step);
    const double bc2 = 1.0 - std::pow(beta2, (double)step);
    AdamArgs a{(float)(1.0 - beta1), (float)beta2, (float)(1.0 - beta2), (float)(lr / bc1), (float)std::sqrt(bc2),
               (float)eps};
    const int64_t n4 = ceil_div(n, (int64_t)4);
    adam_kernel<<<(unsigned)ceil_div(n4, (int64_t)256), 256, 0, as_hip(stream)>>>(param, grad, exp_avg, exp_avg_sq, n,
                                                                                  a);
    LGX_LAUNCH_CHECK();
    return LGX_OK;
}
