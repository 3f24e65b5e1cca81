// C ABI of libmpcd.so (include/mpcd.h): context, weight repacking, schedule -> step plans, and the
// host side of every launch. Host-only code; the kernels live in mlp_sampler.hip,
// cond_prologue.hip, rollout.hip and unet.hip.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <thread>
#include <cmath>
#include <string>
#include <vector>

#include "../../include/mpcd.h"
#include "comm.h"
#include "train.h"

#include <map>
#include "internal.h"
#include "unet.h"

hipError_t launch_clip_flag(const float *x, int64_t n, int *flag_dev, unsigned *ws, hipStream_t stream);
hipError_t launch_unnormalize(const float *x, int64_t n, int dim, const int *flag_dev, const float *mn_host,
                              const float *mx_host, float *out, hipStream_t stream);
hipError_t launch_rollout_cost(const mpcd_system_desc &d, const double *x0_host, const double *x0_dev, int64_t group,
                               const float *u_norm, const float *umin_host, const float *umax_host, const int *flag_dev,
                               int64_t batch, int H, double *cost, hipStream_t stream,
                               const RolloutSelect *sel = nullptr);
hipError_t launch_clip_flags(const float *x, int64_t n_groups, int64_t group_elems, int *flags_dev, hipStream_t stream);
hipError_t launch_normalize_states(const double *x, int64_t M, int C, const float *mn_host, const float *mx_host,
                                   float *out, hipStream_t stream);
hipError_t launch_control_step(const mpcd_system_desc &d, double *x_dev, int64_t M, int64_t group, const float *u_norm,
                               int H, const double *cost, const float *umin_host, const float *umax_host,
                               const int *flags_dev, int select_first, int decimals, double *u_applied,
                               int64_t *best_idx, double *best_cost, hipStream_t stream);
hipError_t launch_argmin(const double *cost, int64_t n, int64_t offset, mpcd_best *best, hipStream_t stream);
hipError_t launch_winner_row(const mpcd_best *best, int64_t lo, int64_t n_local, const float *rows, int row_len,
                             float *out, hipStream_t stream);

int device_cu_count()
{
    constexpr int kMaxDev = 64;
    static std::atomic<int> cu[kMaxDev];  // 0 = not yet queried (zero-initialised: static storage)
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDev) return 256;
    int n = cu[dev].load(std::memory_order_relaxed);
    if (n > 0) return n;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    cu[dev].store(n, std::memory_order_relaxed);
    return n;
}

namespace {

thread_local std::string g_err;

int fail(int code, const char *fmt, ...) __attribute__((format(printf, 2, 3)));
int fail(int code, const char *fmt, ...)
{
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

#define HIP_TRY(expr)                                                                        \
    do {                                                                                     \
        hipError_t e_ = (expr);                                                              \
        if (e_ != hipSuccess) return fail(MPCD_EHIP, "%s: %s", #expr, hipGetErrorString(e_)); \
    } while (0)

// Every entry point runs on its context's device and gives the caller's current device back on return
// (a process driving several GPUs through torch keeps its own current device across our calls).
struct DeviceGuard {
    int prev = -1;
    hipError_t err;
    explicit DeviceGuard(int dev)
    {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        err = prev == dev ? hipSuccess : hipSetDevice(dev);
    }
    ~DeviceGuard()
    {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
    DeviceGuard(const DeviceGuard &) = delete;
    DeviceGuard &operator=(const DeviceGuard &) = delete;
};
#define DEVICE_GUARD(dev)                                                                                 \
    DeviceGuard device_guard_(dev);                                                                       \
    if (device_guard_.err != hipSuccess)                                                                  \
    return fail(MPCD_EHIP, "hipSetDevice(%d): %s", (int)(dev), hipGetErrorString(device_guard_.err))

struct PSpec {
    std::string name;
    std::vector<int64_t> shape;
    int64_t numel() const
    {
        int64_t n = 1;
        for (auto s : shape) n *= s;
        return n;
    }
};

int cond_dim_of(const mpcd_net_desc &d) { return d.time_emb_dim + d.context_dim; }

void add(std::vector<PSpec> &v, const std::string &n, std::vector<int64_t> s) { v.push_back({n, std::move(s)}); }

void time_mlp_spec(std::vector<PSpec> &v, const mpcd_net_desc &d)
{
    add(v, "time_mlp.encoder.1.weight", {128, 32});
    add(v, "time_mlp.encoder.1.bias", {128});
    add(v, "time_mlp.encoder.3.weight", {d.time_emb_dim, 128});
    add(v, "time_mlp.encoder.3.bias", {d.time_emb_dim});
}

// TemporalBlockMLP (layers.py:358-385)
void tbm_spec(std::vector<PSpec> &v, const std::string &p, int ci, int co, int cond)
{
    add(v, p + ".blocks.0._network.0.weight", {co, ci});
    add(v, p + ".blocks.0._network.0.bias", {co});
    add(v, p + ".blocks.0._network.2.weight", {co, co});
    add(v, p + ".blocks.0._network.2.bias", {co});
    add(v, p + ".cond_mlp.1.weight", {co, cond});
    add(v, p + ".cond_mlp.1.bias", {co});
}

// ResidualTemporalBlock (layers.py:323-355)
void rtb_spec(std::vector<PSpec> &v, const std::string &p, int ci, int co, int cond)
{
    add(v, p + ".blocks.0.block.0.weight", {co, ci, 5});
    add(v, p + ".blocks.0.block.0.bias", {co});
    add(v, p + ".blocks.0.block.2.weight", {co});
    add(v, p + ".blocks.0.block.2.bias", {co});
    add(v, p + ".blocks.1.block.0.weight", {co, co, 5});
    add(v, p + ".blocks.1.block.0.bias", {co});
    add(v, p + ".blocks.1.block.2.weight", {co});
    add(v, p + ".blocks.1.block.2.bias", {co});
    add(v, p + ".cond_mlp.1.weight", {co, cond});
    add(v, p + ".cond_mlp.1.bias", {co});
    if (ci != co) {
        add(v, p + ".residual_conv.weight", {co, ci, 1});
        add(v, p + ".residual_conv.bias", {co});
    }
}

std::vector<std::pair<int, int>> stages(int first, const mpcd_net_desc &d)
{
    std::vector<std::pair<int, int>> s;
    int prev = first;
    for (int i = 0; i < d.n_mults; ++i) {
        s.push_back({prev, d.base_dim * d.mults[i]});
        prev = d.base_dim * d.mults[i];
    }
    return s;
}

// state_dict() order of the torch module (registration order: time_mlp, downs, ups, mid, final)
std::vector<PSpec> param_spec(const mpcd_net_desc &d)
{
    std::vector<PSpec> v;
    const int cond = cond_dim_of(d);
    time_mlp_spec(v, d);
    if (d.kind == MPCD_NET_MLP) {
        const int flat = d.horizon * d.state_dim;
        auto st = stages(flat, d);
        for (size_t i = 0; i < st.size(); ++i) tbm_spec(v, "downs." + std::to_string(i) + ".0", st[i].first, st[i].second, cond);
        for (size_t i = 1; i < st.size(); ++i) {
            auto [ci, co] = st[st.size() - i];
            tbm_spec(v, "ups." + std::to_string(i - 1) + ".0", 2 * co, ci, cond);
        }
        const int mid = st.back().second;
        tbm_spec(v, "mid_block1", mid, mid, cond);
        add(v, "final_layer.0._network.0.weight", {d.base_dim, d.base_dim});
        add(v, "final_layer.0._network.0.bias", {d.base_dim});
        add(v, "final_layer.0._network.2.weight", {flat, d.base_dim});
        add(v, "final_layer.0._network.2.bias", {flat});
    } else {
        auto st = stages(d.state_dim, d);
        const int nres = (int)st.size();
        for (int i = 0; i < nres; ++i) {
            const std::string p = "downs." + std::to_string(i);
            rtb_spec(v, p + ".0", st[i].first, st[i].second, cond);
            rtb_spec(v, p + ".1", st[i].second, st[i].second, cond);
            if (i < nres - 1) {
                add(v, p + ".4.conv.weight", {st[i].second, st[i].second, 3});
                add(v, p + ".4.conv.bias", {st[i].second});
            }
        }
        for (int i = 1; i < nres; ++i) {
            auto [ci, co] = st[nres - i];
            const std::string p = "ups." + std::to_string(i - 1);
            rtb_spec(v, p + ".0", 2 * co, ci, cond);
            rtb_spec(v, p + ".1", ci, ci, cond);
            add(v, p + ".4.conv.weight", {ci, ci, 4});
            add(v, p + ".4.conv.bias", {ci});
        }
        const int mid = st.back().second;
        rtb_spec(v, "mid_block1", mid, mid, cond);
        rtb_spec(v, "mid_block2", mid, mid, cond);
        add(v, "final_conv.0.block.0.weight", {d.base_dim, d.base_dim, 5});
        add(v, "final_conv.0.block.0.bias", {d.base_dim});
        add(v, "final_conv.0.block.2.weight", {d.base_dim});
        add(v, "final_conv.0.block.2.bias", {d.base_dim});
        add(v, "final_conv.1.weight", {d.state_dim, d.base_dim, 1});
        add(v, "final_conv.1.bias", {d.state_dim});
    }
    return v;
}

int check_desc(const mpcd_net_desc *d)
{
    if (!d) return fail(MPCD_EINVAL, "null desc");
    if (d->kind != MPCD_NET_MLP && d->kind != MPCD_NET_UNET) return fail(MPCD_EINVAL, "bad net kind %d", d->kind);
    if (d->state_dim < 1 || d->horizon < 1 || d->context_dim < 0 || d->base_dim < 1 || d->n_mults < 1 ||
        d->n_mults > 4 || d->time_emb_dim != 32)
        return fail(MPCD_EINVAL, "bad net dims");
    for (int i = 0; i < d->n_mults; ++i)
        if (d->mults[i] < 1) return fail(MPCD_EINVAL, "bad dim_mults");
    if (d->dtype == MPCD_F16 && d->kind != MPCD_NET_UNET) return fail(MPCD_EUNSUP, "MPCD_F16 is UNet-only");
    if (d->dtype != MPCD_F32 && d->dtype != MPCD_F32X3 && d->dtype != MPCD_F16 && d->dtype != MPCD_F16X2)
        return fail(MPCD_EINVAL, "bad dtype %d", d->dtype);
    return MPCD_OK;
}

struct DevBuf {
    void *p = nullptr;
    size_t bytes = 0;
    int ensure(size_t n)
    {
        if (n <= bytes) return MPCD_OK;
        if (p) (void)hipFree(p);
        p = nullptr;
        bytes = 0;
        if (hipMalloc(&p, n) != hipSuccess) return fail(MPCD_ENOMEM, "hipMalloc(%zu) failed", n);
        bytes = n;
        return MPCD_OK;
    }
    void release()
    {
        if (p) (void)hipFree(p);
        p = nullptr;
        bytes = 0;
    }
    template <class T> T *as() const { return static_cast<T *>(p); }
};

}  // namespace

struct mpcd_ctx {
    int device = 0;
    bool net_loaded = false;
    mpcd_net_desc desc{};
    int cond_dim = 0, cond_total = 0, n_cond = 0;
    DevBuf params;      // raw blob (time MLP, cond layers, UNet tensors)
    DevBuf wpack;       // MLP packed linear layers (fp32 MFMA operand order)
    DevBuf wpack3;      // MLP linear layers split into three bf16 planes (MPCD_F32X3, and MPCD_F16X2's other cases)
    DevBuf wpackh;      // MLP linear layers as two fp16 planes + per-layer scales (MPCD_F16X2)
    DevBuf cond_layers; // CondLayer[n_cond]
    UnetWeights unet{}; // device pointers into `params` + repacked conv weights
    bool force_x3 = false;  // mpcd_force_f32x3: an MPCD_F16X2 net runs its split-bf16 (MPCD_F32X3) programs
    DevBuf unet_pack;
    // schedule
    std::vector<float> tables;  // 12 x N
    std::vector<float> post_std;
    int n_steps = 0;
    // workspace
    DevBuf plan, tproj, cproj, flag, unet_ws;
    std::vector<StepPlan> plan_host;
    // plan + tproj on the device are reused while the plan, net and schedule are unchanged (the
    // time projections do not depend on the context, so a control loop computes them once)
    std::vector<StepPlan> plan_cached;
    bool plan_cached_valid = false;
    hipStream_t plan_stream = nullptr;  // stream the cached plan / tproj were produced on
    hipEvent_t plan_ev = nullptr;       // recorded after they were produced
    // the timing events of the last kEvRing sample calls (ev0 / ev1: the latest pair): a control loop reads the mean
    // kernel time once after its timed steps (mpcd_sample_ms_mean) instead of one host query per step
    static constexpr int kEvRing = 256;
    hipEvent_t evr[2][kEvRing] = {};
    uint32_t ev_n = 0;  // sample calls recorded
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    bool timed = false;
    float *dbg = nullptr;  // debug dump target for mpcd_eps (mpcd_debug_set)
    // candidate-batch data parallelism: one communicator per context (mpcd_comm_init: RCCL;
    // mpcd_comm_init_loopback: virtual ranks on one device)
    Comm *comm = nullptr;
    int nranks = 1, rank = 0;
    // flag: [0] internal clip flag, [16..] zero-initialised counters of the self-resetting reductions
    unsigned *sync_ws() const { return flag.as<unsigned>() + 16; }
    // mpcd_mpc_step: device context row, per-block argmin partials, {best, winner row} result block
    // and its pinned host mirror (one D2H copy per control step)
    DevBuf step_ctx, step_part, step_out, step_amax;
    void *step_host = nullptr;
    void *step_host_dev = nullptr;  // step_host's device address (mapped pinned memory)
    size_t step_host_bytes = 0;
    uint32_t step_seq = 0;          // completion word value of the last single-rank mpcd_mpc_step
    int32_t step_flags = 0;  // mpcd_last_step_flags
};

namespace {

enum {
    T_BETAS = 0, T_AC, T_ACP, T_SQAC, T_SQ1MAC, T_LOG1MAC, T_SRAC, T_SRM1AC, T_PV, T_PLVC, T_C1, T_C2
};

float tab(const mpcd_ctx *c, int which, int t) { return c->tables[(size_t)which * c->n_steps + t]; }

// Build the per-step plan (sample_functions.py:28-44 for DDPM; diffusion_model_base.py:251-290 for DDIM).
int build_plan(mpcd_ctx *c, const mpcd_sample_args *a, std::vector<StepPlan> &plan)
{
    plan.clear();
    const int N = c->n_steps;
    if (a->sampler == MPCD_DDPM_CFG) {
        if (a->n_wo_noise < 0) return fail(MPCD_EINVAL, "n_wo_noise < 0");
        for (int i = N - 1; i >= -a->n_wo_noise; --i) {
            const int t = i < 0 ? 0 : i;
            StepPlan s{};
            s.t = t;
            s.flags = t > 0 ? PLAN_NOISE : 0;
            s.a = tab(c, T_SRAC, t);
            s.b = tab(c, T_SRM1AC, t);
            s.c1 = tab(c, T_C1, t);
            s.c2 = tab(c, T_C2, t);
            s.std = c->post_std[t];
            plan.push_back(s);
        }
        return MPCD_OK;
    }
    // DDIM: times = reversed(int(cat([-1], linspace(0, N-1, S+1)))) unless given explicitly
    std::vector<int> times;
    if (a->ddim_times && a->n_ddim_times > 1) {
        times.assign(a->ddim_times, a->ddim_times + a->n_ddim_times);
    } else {
        const int S = a->ddim_steps > 0 ? a->ddim_steps : N / 5;
        if (S < 1) return fail(MPCD_EINVAL, "DDIM needs at least one sampling step");
        // torch.linspace (fp32, scalar path): start + step*i for i < steps/2, else end - step*(steps-1-i)
        const int steps = S + 1;
        const float start = 0.f, end = (float)(N - 1);
        const float stp = (end - start) / (float)(steps - 1);
        std::vector<int> g;
        for (int i = 0; i < steps; ++i) {
            const float v = i < steps / 2 ? start + stp * (float)i : end - stp * (float)(steps - i - 1);
            g.push_back((int)v);
        }
        times.push_back(-1);
        times.insert(times.end(), g.begin(), g.end());
        std::reverse(times.begin(), times.end());
    }
    for (size_t k = 0; k + 1 < times.size(); ++k) {
        const int t = times[k], tn = times[k + 1];
        if (t < 0 || t >= N || tn >= N) return fail(MPCD_EINVAL, "DDIM time out of range");
        StepPlan s{};
        s.t = t;
        s.a = tab(c, T_SRAC, t);
        s.b = tab(c, T_SRM1AC, t);
        if (tn < 0) {
            s.flags = PLAN_FINAL;
            plan.push_back(s);
            break;
        }
        const float an = tab(c, T_AC, tn);
        s.sqan = sqrtf(an);
        s.cn = sqrtf(1.0f - an - 0.0f);  // sigma = eta * (...) = 0 (eta = 0, :253)
        plan.push_back(s);
    }
    return MPCD_OK;
}

int upload_net(mpcd_ctx *c, const mpcd_net_desc &d, const float *blob, size_t n_floats)
{
    auto spec = param_spec(d);
    size_t total = 0;
    for (auto &p : spec) total += (size_t)p.numel();
    if (n_floats != total) return fail(MPCD_EINVAL, "blob has %zu floats, net needs %zu", n_floats, total);
    std::vector<size_t> off;
    size_t o = 0;
    for (auto &p : spec) {
        off.push_back(o);
        o += (size_t)p.numel();
    }
    auto find = [&](const std::string &n) -> int {
        for (size_t i = 0; i < spec.size(); ++i)
            if (spec[i].name == n) return (int)i;
        return -1;
    };
    int rc = c->params.ensure(total * sizeof(float));
    if (rc) return rc;
    HIP_TRY(hipMemcpy(c->params.p, blob, total * sizeof(float), hipMemcpyHostToDevice));
    const float *dbase = c->params.as<float>();
    auto dptr = [&](const std::string &n) { return dbase + off[find(n)]; };

    // conditioning layers: every "*.cond_mlp.1.weight" in spec order
    std::vector<CondLayer> cl;
    int cond_total = 0;
    for (size_t i = 0; i < spec.size(); ++i) {
        const std::string &n = spec[i].name;
        const std::string suf = ".cond_mlp.1.weight";
        if (n.size() > suf.size() && n.compare(n.size() - suf.size(), suf.size(), suf) == 0) {
            CondLayer L;
            L.W = dbase + off[i];
            L.b = dbase + off[i + 1];
            L.width = (int)spec[i].shape[0];
            L.off = cond_total;
            cond_total += L.width;
            cl.push_back(L);
        }
    }
    if (d.kind == MPCD_NET_MLP) {
        // MLP kernel consumes cond blocks in execution order: downs 0..2, mid, ups 0..1
        // (spec order is downs, ups, mid) -> reorder to execution order and fixed offsets.
        if (cl.size() != 6) return fail(MPCD_EUNSUP, "MLP needs dim_mults of length 3");
        std::vector<CondLayer> ex = {cl[0], cl[1], cl[2], cl[5], cl[3], cl[4]};
        int ofs = 0;
        for (auto &L : ex) {
            L.off = ofs;
            ofs += L.width;
        }
        cl = ex;
        const int d0 = d.horizon * d.state_dim;
        if (d.base_dim != 32 || d.mults[0] != 1 || d.mults[1] != 2 || d.mults[2] != 4 || mlp_packed_floats(d0) < 0)
            return fail(MPCD_EUNSUP, "MLP kernel supports base 32, mults (1,2,4), H*d in {32,64,128}");
        // gather the 14 Linear layers in execution order
        const char *names[14] = {"downs.0.0.blocks.0._network.0", "downs.0.0.blocks.0._network.2",
                                 "downs.1.0.blocks.0._network.0", "downs.1.0.blocks.0._network.2",
                                 "downs.2.0.blocks.0._network.0", "downs.2.0.blocks.0._network.2",
                                 "mid_block1.blocks.0._network.0", "mid_block1.blocks.0._network.2",
                                 "ups.0.0.blocks.0._network.0", "ups.0.0.blocks.0._network.2",
                                 "ups.1.0.blocks.0._network.0", "ups.1.0.blocks.0._network.2",
                                 "final_layer.0._network.0", "final_layer.0._network.2"};
        const float *lw[14], *lb[14];
        for (int l = 0; l < 14; ++l) {
            const int iw = find(std::string(names[l]) + ".weight"), ib = find(std::string(names[l]) + ".bias");
            if (iw < 0 || ib < 0) return fail(MPCD_EINVAL, "missing %s", names[l]);
            lw[l] = blob + off[iw];
            lb[l] = blob + off[ib];
        }
        std::vector<float> packed((size_t)mlp_packed_floats(d0));
        mlp_pack_weights(d0, lw, lb, packed.data());
        rc = c->wpack.ensure(packed.size() * sizeof(float));
        if (rc) return rc;
        HIP_TRY(hipMemcpy(c->wpack.p, packed.data(), packed.size() * sizeof(float), hipMemcpyHostToDevice));
        if (d.dtype == MPCD_F32X3 || d.dtype == MPCD_F16X2) {
            std::vector<float> packed3((size_t)mlp_packed_floats_x3(d0));
            mlp_pack_weights_x3(d0, lw, lb, packed3.data());
            if ((rc = c->wpack3.ensure(packed3.size() * sizeof(float)))) return rc;
            HIP_TRY(hipMemcpy(c->wpack3.p, packed3.data(), packed3.size() * sizeof(float), hipMemcpyHostToDevice));
        }
        if (d.dtype == MPCD_F16X2 && mlp_packed_floats_h2(d0) > 0) {
            std::vector<float> packedh((size_t)mlp_packed_floats_h2(d0));
            mlp_pack_weights_h2(d0, lw, lb, packedh.data());
            if ((rc = c->wpackh.ensure(packedh.size() * sizeof(float)))) return rc;
            HIP_TRY(hipMemcpy(c->wpackh.p, packedh.data(), packedh.size() * sizeof(float), hipMemcpyHostToDevice));
        }
    } else {
        rc = unet_prepare(d, spec.size(), [&](const char *n) -> const float * {
            const int i = find(n);
            return i < 0 ? nullptr : dbase + off[i];
        }, [&](const char *n) -> const float * {
            const int i = find(n);
            return i < 0 ? nullptr : blob + off[i];
        }, c->unet, c->unet_pack.p, c->unet_pack.bytes);
        if (rc) return fail(rc, "unet_prepare: %s", unet_last_error());
    }
    rc = c->cond_layers.ensure(cl.size() * sizeof(CondLayer));
    if (rc) return rc;
    HIP_TRY(hipMemcpy(c->cond_layers.p, cl.data(), cl.size() * sizeof(CondLayer), hipMemcpyHostToDevice));
    c->n_cond = (int)cl.size();
    c->cond_total = cond_total;
    c->cond_dim = cond_dim_of(d);
    c->desc = d;
    c->net_loaded = true;
    return MPCD_OK;
}

}  // namespace

namespace {
// MLP kernel choice (mlp_kernel_of): the two-term fp16 kernel for an MPCD_F16X2 net where it applies (CFG-DDPM or
// the eps forward, H*d 32 / 64, shared context), the split-bf16 kernels for MPCD_F32X3 / the other MPCD_F16X2 cases
// with a shared (or no) context, else the exact-f32 kernel. All are GPU kernels with fp32-level results.
enum { MLPK_F32 = 0, MLPK_X3 = 1, MLPK_H2 = 2 };
int mlp_kernel_of(const mpcd_ctx *c, int mode, bool shared_ctx)
{
    const int d0 = c->desc.horizon * c->desc.state_dim;
    if (c->desc.dtype == MPCD_F16X2 && !c->force_x3 && shared_ctx && c->wpackh.p && mlp_h2_supports(d0, mode))
        return MLPK_H2;
    if ((c->desc.dtype == MPCD_F32X3 || c->desc.dtype == MPCD_F16X2) && shared_ctx) return MLPK_X3;
    return MLPK_F32;
}
hipError_t launch_mlp(mpcd_ctx *c, MlpSampleArgs &m, int nb, hipStream_t st)
{
    const int d0 = c->desc.horizon * c->desc.state_dim;
    const int k = mlp_kernel_of(c, m.mode, m.cproj == nullptr || m.cproj_stride == 0);
    if (k == MLPK_H2) {
        m.wpack = c->wpackh.as<float>();
        const int lay = mlp_x3_layout_of(m.batch, nb);  // the bf16x3 layouts' row choice: 16x8, 16x4, rw16 -> 16 rows
        return launch_mlp_h2(d0, (lay == 1 || lay == 2 || lay == 4) ? 16 : 32, m, st);
    }
    if (k == MLPK_X3) {
        m.wpack = c->wpack3.as<float>();
        return launch_mlp_x3(d0, nb, m, st);
    }
    m.wpack = c->wpack.as<float>();
    return launch_mlp_sampler(d0, nb, m, st);
}
}  // namespace

#ifndef MPCD_SEPARATE_EVENT_RECORDS
#define MPCD_SEPARATE_EVENT_RECORDS 0
#endif
thread_local LaunchEvents g_launch_ev{};

extern "C" {

const char *mpcd_last_error(void) { return g_err.c_str(); }

int mpcd_net_param_count(const mpcd_net_desc *desc, int32_t *n_tensors, int64_t *n_floats)
{
    int rc = check_desc(desc);
    if (rc) return rc;
    auto spec = param_spec(*desc);
    int64_t n = 0;
    for (auto &p : spec) n += p.numel();
    if (n_tensors) *n_tensors = (int32_t)spec.size();
    if (n_floats) *n_floats = n;
    return MPCD_OK;
}

int mpcd_net_param_info(const mpcd_net_desc *desc, int32_t i, char *name, size_t name_cap, int32_t *ndim,
                        int64_t shape[4])
{
    int rc = check_desc(desc);
    if (rc) return rc;
    auto spec = param_spec(*desc);
    if (i < 0 || i >= (int32_t)spec.size()) return fail(MPCD_EINVAL, "tensor index %d out of range", i);
    const PSpec &p = spec[i];
    if (name && name_cap) snprintf(name, name_cap, "%s", p.name.c_str());
    if (ndim) *ndim = (int32_t)p.shape.size();
    if (shape)
        for (size_t k = 0; k < 4; ++k) shape[k] = k < p.shape.size() ? p.shape[k] : 1;
    return MPCD_OK;
}

int mpcd_create(int device, mpcd_ctx **out)
{
    if (!out) return fail(MPCD_EINVAL, "null out");
    int n = 0;
    HIP_TRY(hipGetDeviceCount(&n));
    if (device < 0 || device >= n) return fail(MPCD_EINVAL, "device %d of %d", device, n);
    DEVICE_GUARD(device);
    auto *c = new mpcd_ctx();
    c->device = device;
    bool ev_ok = hipEventCreateWithFlags(&c->plan_ev, hipEventDisableTiming) == hipSuccess;
    for (int i = 0; i < mpcd_ctx::kEvRing && ev_ok; ++i)
        ev_ok = hipEventCreate(&c->evr[0][i]) == hipSuccess && hipEventCreate(&c->evr[1][i]) == hipSuccess;
    if (!ev_ok) {
        for (int i = 0; i < mpcd_ctx::kEvRing; ++i)
            for (int j = 0; j < 2; ++j)
                if (c->evr[j][i]) (void)hipEventDestroy(c->evr[j][i]);
        if (c->plan_ev) (void)hipEventDestroy(c->plan_ev);
        delete c;
        return fail(MPCD_EHIP, "hipEventCreate failed");
    }
    c->ev0 = c->evr[0][0];
    c->ev1 = c->evr[1][0];
    if (int rc = c->flag.ensure(256)) {
        delete c;
        return rc;
    }
    if (hipMemset(c->flag.p, 0, 256) != hipSuccess || hipDeviceSynchronize() != hipSuccess) {
        c->flag.release();
        delete c;
        return fail(MPCD_EHIP, "hipMemset of the reduction counters failed");
    }
    *out = c;
    return MPCD_OK;
}

void mpcd_destroy(mpcd_ctx *c)
{
    if (!c) return;
    DeviceGuard device_guard_(c->device);
    for (DevBuf *b : {&c->params, &c->wpack, &c->wpack3, &c->wpackh, &c->cond_layers, &c->unet_pack, &c->plan, &c->tproj, &c->cproj, &c->flag,
                      &c->unet_ws, &c->step_ctx, &c->step_part, &c->step_out, &c->step_amax})
        b->release();
    for (int i = 0; i < mpcd_ctx::kEvRing; ++i)
        for (int j = 0; j < 2; ++j)
            if (c->evr[j][i]) (void)hipEventDestroy(c->evr[j][i]);
    if (c->plan_ev) (void)hipEventDestroy(c->plan_ev);
    delete c->comm;
    if (c->step_host) (void)hipHostFree(c->step_host);
    delete c;
}

int mpcd_load_net(mpcd_ctx *c, const mpcd_net_desc *desc, const float *blob, size_t n_floats)
{
    if (!c || !blob) return fail(MPCD_EINVAL, "null argument");
    int rc = check_desc(desc);
    if (rc) return rc;
    DEVICE_GUARD(c->device);
    c->net_loaded = false;
    c->plan_cached_valid = false;
    return upload_net(c, *desc, blob, n_floats);
}

int mpcd_set_schedule(mpcd_ctx *c, const float *tables, int32_t n_steps, const float *post_std)
{
    if (!c || !tables || n_steps < 1) return fail(MPCD_EINVAL, "bad schedule arguments");
    c->tables.assign(tables, tables + (size_t)12 * n_steps);
    c->post_std.resize(n_steps);
    for (int t = 0; t < n_steps; ++t)
        c->post_std[t] = post_std ? post_std[t] : sqrtf(expf(tables[(size_t)T_PLVC * n_steps + t]));
    c->n_steps = n_steps;
    c->plan_cached_valid = false;
    return MPCD_OK;
}

int mpcd_sample_steps(mpcd_ctx *c, const mpcd_sample_args *a, int32_t *n)
{
    if (!c || !a || !n) return fail(MPCD_EINVAL, "null argument");
    if (!c->n_steps) return fail(MPCD_ESTATE, "no schedule set");
    std::vector<StepPlan> plan;
    int rc = build_plan(c, a, plan);
    if (rc) return rc;
    *n = (int32_t)plan.size();
    return MPCD_OK;
}

// ctx_row: mpcd_mpc_step's one shared context row by value (the ctx prologue reads it from its kernel
// arguments: no host-to-device copy); nullptr: a->context on the device (the C-ABI mpcd_sample)
static int sample_impl(mpcd_ctx *c, const mpcd_sample_args *a, void *stream_ptr, const CtxRowArg *ctx_row);

int mpcd_sample(mpcd_ctx *c, const mpcd_sample_args *a, void *stream_ptr)
{
    return sample_impl(c, a, stream_ptr, nullptr);
}

static int sample_impl(mpcd_ctx *c, const mpcd_sample_args *a, void *stream_ptr, const CtxRowArg *ctx_row)
{
    if (!c || !a) return fail(MPCD_EINVAL, "null argument");
    if (!c->net_loaded) return fail(MPCD_ESTATE, "no net loaded");
    if (!c->n_steps) return fail(MPCD_ESTATE, "no schedule set");
    if (!a->x_out || a->batch < 1) return fail(MPCD_EINVAL, "x_out / batch");
    const mpcd_net_desc &d = c->desc;
    const bool cfg = a->sampler == MPCD_DDPM_CFG || a->sampler == MPCD_DDIM_CFG;
    if (a->sampler < 0 || a->sampler > MPCD_DDIM) return fail(MPCD_EINVAL, "bad sampler %d", a->sampler);
    if (cfg != (d.cfg_masked != 0)) return fail(MPCD_EINVAL, "CFG samplers need a cfg_masked net and vice versa");
    if (d.context_dim > 0 && !a->context && !ctx_row) return fail(MPCD_EINVAL, "net has a context but none given");
    hipStream_t st = static_cast<hipStream_t>(stream_ptr);
    DEVICE_GUARD(c->device);

    int rc = build_plan(c, a, c->plan_host);
    if (rc) return rc;
    const int S = (int)c->plan_host.size();
    const CondLayer *cl = c->cond_layers.as<CondLayer>();
    const bool reuse = c->plan_cached_valid && c->plan_cached.size() == c->plan_host.size() &&
                       memcmp(c->plan_cached.data(), c->plan_host.data(), sizeof(StepPlan) * S) == 0;
    if (!reuse) {
        if ((rc = c->plan.ensure(sizeof(StepPlan) * S))) return rc;
        HIP_TRY(hipMemcpyAsync(c->plan.p, c->plan_host.data(), sizeof(StepPlan) * S, hipMemcpyHostToDevice, st));
        if ((rc = c->tproj.ensure(sizeof(float) * (size_t)S * c->cond_total))) return rc;
        const float *P = c->params.as<float>();
        // time MLP = the first four tensors of the blob
        const float *tw1 = P, *tb1 = tw1 + 128 * 32, *tw2 = tb1 + 128, *tb2 = tw2 + 32 * 128;
        launch_time_prologue(c->plan.as<StepPlan>(), S, tw1, tb1, tw2, tb2, cl, c->n_cond, c->cond_dim, c->cond_total,
                             c->tproj.as<float>(), st);
        HIP_TRY(hipGetLastError());
        c->plan_cached = c->plan_host;
        c->plan_cached_valid = true;
        c->plan_stream = st;
        HIP_TRY(hipEventRecord(c->plan_ev, st));
    } else if (st != c->plan_stream) {  // cached plan / tproj were written on another stream
        HIP_TRY(hipStreamWaitEvent(st, c->plan_ev, 0));
    }
    const float *cproj = nullptr;
    int64_t cstride = 0;
    // the MLP samplers with a shared context (fp16 two-term and split-bf16; not the exact-f32 kernel, which stages
    // per-candidate projections) compute mpcd_mpc_step's row projection in their own staging: one launch fewer
    const int mk = d.kind == MPCD_NET_MLP ? mlp_kernel_of(c, a->sampler, true) : -1;
    const bool fuse_ctx = ctx_row && (mk == MLPK_H2 || mk == MLPK_X3);
    if (d.context_dim > 0) {
        const bool shared = ctx_row || a->context_shared;
        const int64_t rows = shared ? 1 : a->batch;
        if ((rc = c->cproj.ensure(sizeof(float) * (size_t)rows * c->cond_total))) return rc;
        if (fuse_ctx) {
            // computed by the sampler launch itself (ctx_proj_col)
        } else if (ctx_row)
            launch_ctx_prologue_row(*ctx_row, d.context_dim, cl, c->n_cond, c->cond_dim, c->cond_total,
                                    c->cproj.as<float>(), st);
        else
            launch_ctx_prologue(a->context, rows, d.context_dim, cl, c->n_cond, c->cond_dim, c->cond_total,
                                c->cproj.as<float>(), st);
        HIP_TRY(hipGetLastError());
        cproj = c->cproj.as<float>();
        cstride = shared ? 0 : c->cond_total;
    }
    const float wp1 = (float)(1.0 + a->w), wf = (float)a->w;
    c->ev0 = c->evr[0][c->ev_n % mpcd_ctx::kEvRing];
    c->ev1 = c->evr[1][c->ev_n % mpcd_ctx::kEvRing];
    // the MLP sampler's launch records both events itself (MPCD_SEPARATE_EVENT_RECORDS: separate records, A/B build)
    constexpr bool kExtEv = !MPCD_SEPARATE_EVENT_RECORDS;
    if (d.kind != MPCD_NET_MLP || !kExtEv) HIP_TRY(hipEventRecord(c->ev0, st));
    if (d.kind == MPCD_NET_MLP) {
        MlpSampleArgs m{};
        m.dbg = c->dbg;  // read only by the MPCD_PROF_LAYERS experiment build
        m.wpack = c->wpack.as<float>();
        m.plan = c->plan.as<StepPlan>();
        m.tproj = c->tproj.as<float>();
        m.cproj = cproj;
        m.cproj_stride = cstride;
        m.noise = a->noise;
        m.x_out = a->x_out;
        m.chain = a->chain_out;
        m.chain_absmax = a->chain_absmax;
        m.batch = a->batch;
        m.global_offset = a->global_offset;
        m.seed = a->seed;
        m.n_steps = S;
        m.mode = a->sampler;
        m.clamp_x0 = a->clamp_x0;
        m.wp1 = wp1;
        m.wf = wf;
        if (fuse_ctx) {
            m.ctx_fused = 1;
            m.ctx_row = *ctx_row;
            m.ctx_dim = d.context_dim;
            m.cond_layers = cl;
            m.n_cond = c->n_cond;
            m.cond_dim = c->cond_dim;
        }
        if (kExtEv) g_launch_ev = LaunchEvents{c->ev0, c->ev1};
        const hipError_t le = launch_mlp(c, m, cfg ? 2 : 1, st);
        g_launch_ev = LaunchEvents{};
        HIP_TRY(le);
    } else {
        UnetSampleArgs u{};
        u.plan = c->plan.as<StepPlan>();
        u.plan_host = c->plan_host.data();
        u.tproj = c->tproj.as<float>();
        u.cproj = cproj;
        u.cproj_stride = cstride;
        u.cond_total = c->cond_total;
        u.noise = a->noise;
        u.x_out = a->x_out;
        u.chain = a->chain_out;
        u.chain_absmax = a->chain_absmax;
        u.batch = a->batch;
        u.global_offset = a->global_offset;
        u.seed = a->seed;
        u.n_steps = S;
        u.mode = a->sampler;
        u.clamp_x0 = a->clamp_x0;
        u.wp1 = wp1;
        u.wf = wf;
        u.fused = unet_use_fused(c->unet, u.mode);  // once: sizes the workspace and picks the kernels
        size_t ws = unet_workspace_bytes(d, c->unet, u.fused, a->batch, cfg ? 2 : 1);
        if ((rc = c->unet_ws.ensure(ws))) return rc;
        u.workspace = c->unet_ws.p;
        rc = unet_sample(d, c->unet, u, st);
        if (rc) return fail(rc, "unet_sample: %s", unet_last_error());
    }
    if (d.kind != MPCD_NET_MLP || !kExtEv) HIP_TRY(hipEventRecord(c->ev1, st));
    c->timed = true;
    ++c->ev_n;
    return MPCD_OK;
}

int mpcd_eps(mpcd_ctx *c, const float *x, int32_t t, const float *context, int32_t context_shared, int64_t batch,
             float *eps_cond, float *eps_uncond, void *stream_ptr)
{
    if (!c || !x || !eps_cond || batch < 1) return fail(MPCD_EINVAL, "bad mpcd_eps arguments");
    if (!c->net_loaded) return fail(MPCD_ESTATE, "no net loaded");
    if (!c->n_steps) return fail(MPCD_ESTATE, "no schedule set");
    const mpcd_net_desc &d = c->desc;
    const bool cfg = d.cfg_masked != 0;
    if (cfg && !eps_uncond) return fail(MPCD_EINVAL, "cfg net needs eps_uncond");
    if (d.context_dim > 0 && !context) return fail(MPCD_EINVAL, "net has a context but none given");
    if (t < 0 || t >= c->n_steps) return fail(MPCD_EINVAL, "t out of range");
    hipStream_t st = static_cast<hipStream_t>(stream_ptr);
    DEVICE_GUARD(c->device);
    StepPlan sp{};
    sp.t = t;
    c->plan_host.assign(1, sp);
    c->plan_cached_valid = false;  // plan and tproj are overwritten below
    int rc;
    if ((rc = c->plan.ensure(sizeof(StepPlan)))) return rc;
    HIP_TRY(hipMemcpyAsync(c->plan.p, c->plan_host.data(), sizeof(StepPlan), hipMemcpyHostToDevice, st));
    if ((rc = c->tproj.ensure(sizeof(float) * (size_t)c->cond_total))) return rc;
    const CondLayer *cl = c->cond_layers.as<CondLayer>();
    const float *P = c->params.as<float>();
    launch_time_prologue(c->plan.as<StepPlan>(), 1, P, P + 128 * 32, P + 128 * 32 + 128, P + 128 * 32 + 128 + 32 * 128,
                         cl, c->n_cond, c->cond_dim, c->cond_total, c->tproj.as<float>(), st);
    const float *cproj = nullptr;
    int64_t cstride = 0;
    if (d.context_dim > 0) {
        const int64_t rows = context_shared ? 1 : batch;
        if ((rc = c->cproj.ensure(sizeof(float) * (size_t)rows * c->cond_total))) return rc;
        launch_ctx_prologue(context, rows, d.context_dim, cl, c->n_cond, c->cond_dim, c->cond_total,
                            c->cproj.as<float>(), st);
        cproj = c->cproj.as<float>();
        cstride = context_shared ? 0 : c->cond_total;
    }
    if (d.kind == MPCD_NET_UNET) {
        UnetSampleArgs u{};
        u.plan = c->plan.as<StepPlan>();
        u.tproj = c->tproj.as<float>();
        u.cproj = cproj;
        u.cproj_stride = cstride;
        u.cond_total = c->cond_total;
        u.batch = batch;
        u.n_steps = 1;
        u.mode = cfg ? MODE_EPS : MODE_EPS1;
        u.x_in = x;
        u.eps_cond = eps_cond;
        u.eps_uncond = eps_uncond;
        u.fused = unet_use_fused(c->unet, u.mode);
        if ((rc = c->unet_ws.ensure(unet_workspace_bytes(d, c->unet, u.fused, batch, cfg ? 2 : 1)))) return rc;
        u.workspace = c->unet_ws.p;
        rc = unet_sample(d, c->unet, u, st);
        if (rc) return fail(rc, "unet eps: %s", unet_last_error());
        return MPCD_OK;
    }
    MlpSampleArgs m{};
    m.wpack = c->wpack.as<float>();
    m.plan = c->plan.as<StepPlan>();
    m.tproj = c->tproj.as<float>();
    m.cproj = cproj;
    m.cproj_stride = cstride;
    m.noise = x;
    m.x_out = eps_cond;
    m.chain = eps_uncond;
    m.batch = batch;
    m.n_steps = 1;
    m.mode = cfg ? MODE_EPS : MODE_EPS1;
    m.dbg = c->dbg;
    HIP_TRY(launch_mlp(c, m, cfg ? 2 : 1, st));
    return MPCD_OK;
}

int mpcd_philox_noise(uint64_t seed, int64_t global_offset, int64_t n_cand, int32_t n_slices, int32_t flat,
                      float *out, void *stream)
{
    if (!out || n_cand < 1 || n_slices < 1 || flat < 4 || flat % 4 || global_offset < 0)
        return fail(MPCD_EINVAL, "bad mpcd_philox_noise arguments");
    HIP_TRY(launch_philox_noise(seed, global_offset, n_cand, n_slices, flat, out, static_cast<hipStream_t>(stream)));
    return MPCD_OK;
}

int mpcd_last_step_flags(mpcd_ctx *c, int32_t *flags)
{
    if (!c || !flags) return fail(MPCD_EINVAL, "null argument");
    *flags = c->step_flags;
    return MPCD_OK;
}

int mpcd_unet_force_tiling(int32_t conv_pick, int32_t block_pick)
{
    if (conv_pick < -1 || block_pick < -2) return fail(MPCD_EINVAL, "conv_pick >= -1, block_pick >= -2");
    unet_force_tiling(conv_pick, block_pick);
    return MPCD_OK;
}

int mpcd_unet_force_path(int32_t path)
{
    if (path < 0 || path > 2) return fail(MPCD_EINVAL, "path 0 (auto), 1 (layer by layer) or 2 (fused)");
    unet_force_path(path);
    return MPCD_OK;
}

int mpcd_unet_form(mpcd_ctx *c, int32_t sampler, int32_t out[4])
{
    if (!c || !out) return fail(MPCD_EINVAL, "null argument");
    if (c->desc.kind != MPCD_NET_UNET) return fail(MPCD_EUNSUP, "not a U-Net context");
    if (sampler < MPCD_DDPM_CFG || sampler > MPCD_DDIM) return fail(MPCD_EINVAL, "bad sampler %d", sampler);
    if (!c->unet.ready) return fail(MPCD_ESTATE, "U-Net parameters not loaded");
    unet_form(c->unet, sampler, out);
    return MPCD_OK;
}

int mpcd_mlp_form(mpcd_ctx *c, int32_t sampler, int64_t batch, int32_t out[3])
{
    if (!c || !out || batch < 1) return fail(MPCD_EINVAL, "bad argument");
    if (!c->net_loaded || c->desc.kind != MPCD_NET_MLP) return fail(MPCD_EUNSUP, "not an MLP context");
    if (sampler < MPCD_DDPM_CFG || sampler > MPCD_DDIM) return fail(MPCD_EINVAL, "bad sampler %d", sampler);
    DEVICE_GUARD(c->device);
    const int nb = c->desc.cfg_masked ? 2 : 1;
    const int lay = mlp_x3_layout_of(batch, nb);
    const int k = mlp_kernel_of(c, sampler, true);
    out[0] = k;
    out[1] = k == MLPK_X3 ? lay : -1;
    out[2] = (lay == 1 || lay == 2 || lay == 4) ? 16 : 32;
    return MPCD_OK;
}

int mpcd_force_f32x3(mpcd_ctx *c, int32_t on)
{
    if (!c) return fail(MPCD_EINVAL, "null context");
    c->force_x3 = on != 0;
    c->unet.force3 = on != 0;
    return MPCD_OK;
}

int mpcd_mlp_layout(int64_t batch, int32_t cfg_masked, int32_t *layout_out)
{
    if (batch < 1 || !layout_out) return fail(MPCD_EINVAL, "mpcd_mlp_layout: bad arguments");
    *layout_out = mlp_x3_layout_of(batch, cfg_masked ? 2 : 1);
    return MPCD_OK;
}

int mpcd_mlp_force_layout(int32_t layout)
{
    if (layout < -1 || layout > 4)
        return fail(MPCD_EINVAL, "layout -1 (auto), 0 (32x8), 1 (16x8), 2 (16x4), 3 (rw32) or 4 (rw16)");
    mlp_x3_force_layout(layout);
    return MPCD_OK;
}

int mpcd_last_sample_ms(mpcd_ctx *c, float *ms)
{
    if (!c || !ms) return fail(MPCD_EINVAL, "null argument");
    if (!c->timed) return fail(MPCD_ESTATE, "no sample call recorded");
    HIP_TRY(hipEventSynchronize(c->ev1));
    HIP_TRY(hipEventElapsedTime(ms, c->ev0, c->ev1));
    return MPCD_OK;
}

int mpcd_sample_ms_mean(mpcd_ctx *c, int32_t n, float *ms)
{
    if (!c || !ms) return fail(MPCD_EINVAL, "null argument");
    if (n < 1 || (uint32_t)n > c->ev_n || n > mpcd_ctx::kEvRing)
        return fail(MPCD_EINVAL, "mpcd_sample_ms_mean: %d calls asked, %u recorded, at most %d kept", n, c->ev_n,
                    mpcd_ctx::kEvRing);
    HIP_TRY(hipEventSynchronize(c->ev1));
    double sum = 0.0;
    for (int k = 0; k < n; ++k) {
        const int i = (int)((c->ev_n - 1 - (uint32_t)k) % mpcd_ctx::kEvRing);
        float t = 0.f;
        HIP_TRY(hipEventElapsedTime(&t, c->evr[0][i], c->evr[1][i]));
        sum += t;
    }
    *ms = (float)(sum / n);
    return MPCD_OK;
}

// Not in mpcd.h: debug / profiling dump target (layer activations in mpcd_eps, per-layer cycles in
// the MPCD_PROF_LAYERS experiment build). Null disables.
int mpcd_debug_set(mpcd_ctx *c, float *dbg)
{
    if (!c) return fail(MPCD_EINVAL, "null argument");
    c->dbg = dbg;
    return MPCD_OK;
}

int mpcd_clip_flag(mpcd_ctx *c, const float *x, int64_t n, int32_t *flag, void *stream_ptr)
{
    if (!c || !x || !flag || n < 1) return fail(MPCD_EINVAL, "bad clip_flag arguments");
    DEVICE_GUARD(c->device);
    HIP_TRY(launch_clip_flag(x, n, flag, c->sync_ws(), static_cast<hipStream_t>(stream_ptr)));
    return MPCD_OK;
}

int mpcd_rollout_cost(mpcd_ctx *c, const mpcd_system_desc *sys, const double *x0, const float *u_norm,
                      const float *umin, const float *umax, int64_t batch, int32_t horizon, const int32_t *clip_flag,
                      double *cost, void *stream_ptr)
{
    if (!c || !sys || !x0 || !u_norm || !umin || !umax || !cost) return fail(MPCD_EINVAL, "null argument");
    if (batch < 1 || horizon < 2) return fail(MPCD_EINVAL, "batch/horizon");
    if (sys->n_x < 1 || sys->n_x > 12 || sys->n_u < 1 || sys->n_u > 4) return fail(MPCD_EINVAL, "n_x/n_u");
    if (sys->system < 0 || sys->system > MPCD_SYS_QUADROTOR12) return fail(MPCD_EINVAL, "system %d", sys->system);
    if (sys->cost_kind == MPCD_COST_CALMPC && (sys->n_u != 1 || horizon < 3))
        return fail(MPCD_EINVAL, "calMPCCost needs n_u == 1 and H >= 3");
    if ((size_t)horizon * sys->n_u * 64 * sizeof(float) > 64 * 1024) return fail(MPCD_EUNSUP, "H*n_u too large");
    hipStream_t st = static_cast<hipStream_t>(stream_ptr);
    DEVICE_GUARD(c->device);
    const int *flag = clip_flag;
    if (!flag) {
        HIP_TRY(launch_clip_flag(u_norm, batch * horizon * sys->n_u, c->flag.as<int>(), c->sync_ws(), st));
        flag = c->flag.as<int>();
    }
    HIP_TRY(launch_rollout_cost(*sys, x0, nullptr, batch, u_norm, umin, umax, flag, batch, horizon, cost, st));
    return MPCD_OK;
}

namespace {
int check_system(const mpcd_system_desc *sys, int32_t horizon)
{
    if (sys->n_x < 1 || sys->n_x > 12 || sys->n_u < 1 || sys->n_u > 4) return fail(MPCD_EINVAL, "n_x/n_u");
    if (sys->system < 0 || sys->system > MPCD_SYS_QUADROTOR12) return fail(MPCD_EINVAL, "system %d", sys->system);
    if (sys->cost_kind == MPCD_COST_CALMPC && (sys->n_u != 1 || horizon < 3))
        return fail(MPCD_EINVAL, "calMPCCost needs n_u == 1 and H >= 3");
    if ((size_t)horizon * sys->n_u * 64 * sizeof(float) > 64 * 1024) return fail(MPCD_EUNSUP, "H*n_u too large");
    return MPCD_OK;
}
}  // namespace

int mpcd_clip_flags(mpcd_ctx *c, const float *x, int64_t n_groups, int64_t group_elems, int32_t *flags, void *stream_ptr)
{
    if (!c || !x || !flags) return fail(MPCD_EINVAL, "null argument");
    if (n_groups < 1 || group_elems < 1) return fail(MPCD_EINVAL, "n_groups / group_elems");
    DEVICE_GUARD(c->device);
    HIP_TRY(launch_clip_flags(x, n_groups, group_elems, flags, static_cast<hipStream_t>(stream_ptr)));
    return MPCD_OK;
}

int mpcd_normalize_states(mpcd_ctx *c, const double *x, int64_t n_states, int32_t dim, const float *mn,
                          const float *mx, float *out, void *stream_ptr)
{
    if (!c || !x || !mn || !mx || !out) return fail(MPCD_EINVAL, "null argument");
    if (n_states < 1 || dim < 1 || dim > 16) return fail(MPCD_EINVAL, "n_states / dim (1..16)");
    DEVICE_GUARD(c->device);
    HIP_TRY(launch_normalize_states(x, n_states, dim, mn, mx, out, static_cast<hipStream_t>(stream_ptr)));
    return MPCD_OK;
}

int mpcd_rollout_cost_grouped(mpcd_ctx *c, const mpcd_system_desc *sys, const double *x0_dev, int64_t group,
                              const float *u_norm, const float *umin, const float *umax, int64_t batch,
                              int32_t horizon, const int32_t *flags, double *cost, void *stream_ptr)
{
    if (!c || !sys || !x0_dev || !u_norm || !umin || !umax || !flags || !cost) return fail(MPCD_EINVAL, "null argument");
    if (batch < 1 || horizon < 2 || group < 1 || batch % group) return fail(MPCD_EINVAL, "batch/group/horizon");
    int rc = check_system(sys, horizon);
    if (rc) return rc;
    DEVICE_GUARD(c->device);
    HIP_TRY(launch_rollout_cost(*sys, nullptr, x0_dev, group, u_norm, umin, umax, flags, batch, horizon, cost,
                                static_cast<hipStream_t>(stream_ptr)));
    return MPCD_OK;
}

int mpcd_control_step(mpcd_ctx *c, const mpcd_system_desc *sys, double *x, int64_t n_states, int64_t group,
                      const float *u_norm, int32_t horizon, const double *cost, const float *umin, const float *umax,
                      const int32_t *flags, int32_t select_first, int32_t decimals, double *u_applied,
                      int64_t *best_index, double *best_cost, void *stream_ptr)
{
    if (!c || !sys || !x || !u_norm || !cost || !umin || !umax || !flags || !u_applied || !best_index || !best_cost)
        return fail(MPCD_EINVAL, "null argument");
    if (n_states < 1 || group < 1 || horizon < 1) return fail(MPCD_EINVAL, "n_states/group/horizon");
    if (decimals > 15) return fail(MPCD_EINVAL, "decimals > 15");
    int rc = check_system(sys, horizon);
    if (rc) return rc;
    DEVICE_GUARD(c->device);
    HIP_TRY(launch_control_step(*sys, x, n_states, group, u_norm, horizon, cost, umin, umax, flags, select_first,
                                decimals, u_applied, best_index, best_cost, static_cast<hipStream_t>(stream_ptr)));
    return MPCD_OK;
}

int mpcd_unnormalize(mpcd_ctx *c, const float *x, int64_t n_rows, int32_t dim, const float *mn, const float *mx,
                     const int32_t *clip_flag, float *out, void *stream_ptr)
{
    if (!c || !x || !mn || !mx || !out) return fail(MPCD_EINVAL, "null argument");
    if (dim < 1 || dim > 16 || n_rows < 1) return fail(MPCD_EINVAL, "dim must be 1..16");
    hipStream_t st = static_cast<hipStream_t>(stream_ptr);
    DEVICE_GUARD(c->device);
    const int *flag = clip_flag;
    if (!flag) {
        HIP_TRY(launch_clip_flag(x, n_rows * dim, c->flag.as<int>(), c->sync_ws(), st));
        flag = c->flag.as<int>();
    }
    HIP_TRY(launch_unnormalize(x, n_rows * dim, dim, flag, mn, mx, out, st));
    return MPCD_OK;
}

int mpcd_argmin(mpcd_ctx *c, const double *cost, int64_t n, int64_t offset, mpcd_best *best, void *stream_ptr)
{
    if (!c || !cost || !best || n < 1) return fail(MPCD_EINVAL, "bad argmin arguments");
    hipStream_t st = static_cast<hipStream_t>(stream_ptr);
    DEVICE_GUARD(c->device);
    HIP_TRY(launch_argmin(cost, n, offset, best, st));
    return MPCD_OK;
}

// ---- candidate-batch data parallelism over RCCL

int mpcd_comm_unique_id(void *id_out)
{
    if (!id_out) return fail(MPCD_EINVAL, "null argument");
    std::string e;
    int rc = comm_unique_id(id_out, e);
    return rc ? fail(rc, "%s", e.c_str()) : MPCD_OK;
}

int mpcd_comm_init(mpcd_ctx *c, int32_t nranks, int32_t rank, const void *id_in)
{
    if (!c || !id_in || nranks < 1 || rank < 0 || rank >= nranks) return fail(MPCD_EINVAL, "bad comm arguments");
    if (c->comm) return fail(MPCD_ESTATE, "communicator already initialised");
    DEVICE_GUARD(c->device);
    std::string e;
    int rc = comm_create_rccl(nranks, rank, id_in, &c->comm, e);
    if (rc) return fail(rc, "%s", e.c_str());
    c->nranks = nranks;
    c->rank = rank;
    return MPCD_OK;
}

int mpcd_comm_init_loopback(mpcd_ctx *c, int32_t nranks, int32_t rank, uint64_t group_key)
{
    if (!c || nranks < 1 || rank < 0 || rank >= nranks) return fail(MPCD_EINVAL, "bad comm arguments");
    if (c->comm) return fail(MPCD_ESTATE, "communicator already initialised");
    DEVICE_GUARD(c->device);
    std::string e;
    int rc = comm_create_loopback(nranks, rank, group_key, &c->comm, e);
    if (rc) return fail(rc, "%s", e.c_str());
    c->nranks = nranks;
    c->rank = rank;
    return MPCD_OK;
}

int mpcd_comm_info(mpcd_ctx *c, int32_t *nranks, int32_t *rank)
{
    if (!c || !nranks || !rank) return fail(MPCD_EINVAL, "null argument");
    *nranks = c->nranks;
    *rank = c->rank;
    return MPCD_OK;
}

static int comm_gather(mpcd_ctx *c, const void *send, void *recv, size_t count, size_t esz, hipStream_t st)
{
    DEVICE_GUARD(c->device);
    if (!c->comm) {  // single rank: the gather is a copy
        if (send != recv) HIP_TRY(hipMemcpyAsync(recv, send, count * esz, hipMemcpyDeviceToDevice, st));
        return MPCD_OK;
    }
    std::string e;
    int rc = c->comm->allgather(send, recv, count * esz, st, e);
    return rc ? fail(rc, "allgather: %s", e.c_str()) : MPCD_OK;
}

static int comm_reduce(mpcd_ctx *c, void *buf, size_t count, CommOp op, hipStream_t st)
{
    if (!c->comm) return MPCD_OK;
    std::string e;
    int rc = c->comm->allreduce(buf, count, op, st, e);
    return rc ? fail(rc, "allreduce: %s", e.c_str()) : MPCD_OK;
}

int mpcd_allgather_f32(mpcd_ctx *c, const float *send, float *recv, size_t count_per_rank, void *stream)
{
    if (!c || !send || !recv) return fail(MPCD_EINVAL, "null argument");
    return comm_gather(c, send, recv, count_per_rank, 4, static_cast<hipStream_t>(stream));
}

int mpcd_allgather_f64(mpcd_ctx *c, const double *send, double *recv, size_t count_per_rank, void *stream)
{
    if (!c || !send || !recv) return fail(MPCD_EINVAL, "null argument");
    return comm_gather(c, send, recv, count_per_rank, 8, static_cast<hipStream_t>(stream));
}

int mpcd_broadcast_f32(mpcd_ctx *c, float *buf, size_t count, int32_t root, void *stream)
{
    if (!c || !buf || root < 0 || root >= c->nranks) return fail(MPCD_EINVAL, "bad broadcast arguments");
    DEVICE_GUARD(c->device);
    if (!c->comm) return MPCD_OK;
    std::string e;
    int rc = c->comm->broadcast(buf, count * 4, root, static_cast<hipStream_t>(stream), e);
    return rc ? fail(rc, "broadcast: %s", e.c_str()) : MPCD_OK;
}

int mpcd_allreduce_max_i32(mpcd_ctx *c, int32_t *buf, size_t count, void *stream)
{
    if (!c || !buf) return fail(MPCD_EINVAL, "null argument");
    DEVICE_GUARD(c->device);
    return comm_reduce(c, buf, count, COMM_MAX_I32, static_cast<hipStream_t>(stream));
}

int mpcd_select(mpcd_ctx *c, const double *cost_local, int64_t n_local, const float *rows_local, int32_t row_len,
                double *costs_all, mpcd_best *best_dev, float *row_out, void *stream)
{
    if (!c || !cost_local || !rows_local || !costs_all || !best_dev || !row_out || n_local < 1 || row_len < 1)
        return fail(MPCD_EINVAL, "bad select arguments");
    hipStream_t st = static_cast<hipStream_t>(stream);
    int rc = comm_gather(c, cost_local, costs_all, (size_t)n_local, 8, st);
    if (rc) return rc;
    HIP_TRY(launch_argmin(costs_all, n_local * c->nranks, 0, best_dev, st));
    HIP_TRY(launch_winner_row(best_dev, (int64_t)c->rank * n_local, n_local, rows_local, row_len, row_out, st));
    return comm_reduce(c, row_out, (size_t)row_len, COMM_SUM_F32, st);
}

static int mpc_step_impl(mpcd_ctx *c, const mpcd_step_args *a, mpcd_best *best_host, float *u_best_host, void *stream);

// An MPCD_F16X2 net computes in the fp16 range: a step whose sampled trajectories came back with a NaN (an
// activation beyond 65504 turns into one: hi = inf, lo = inf - inf) or with no finite cost is re-run with the net's
// split-bf16 (MPCD_F32X3) programs and flagged MPCD_STEP_F32X3_RERUN. Single rank only: with a communicator every
// rank would have to agree to re-run (the flag and the ENONFINITE return report it there).
int mpcd_mpc_step(mpcd_ctx *c, const mpcd_step_args *a, mpcd_best *best_host, float *u_best_host, void *stream)
{
    int rc = mpc_step_impl(c, a, best_host, u_best_host, stream);
    const bool f16x2 = c && c->net_loaded && c->desc.dtype == MPCD_F16X2 && !c->force_x3;
    if (f16x2 && !c->comm && (rc == MPCD_ENONFINITE || (rc == MPCD_OK && (c->step_flags & MPCD_STEP_NAN_SAMPLES)))) {
        c->force_x3 = c->unet.force3 = true;
        rc = mpc_step_impl(c, a, best_host, u_best_host, stream);
        c->force_x3 = c->unet.force3 = false;
        c->step_flags |= MPCD_STEP_F32X3_RERUN;
    }
    return rc;
}

static int mpc_step_impl(mpcd_ctx *c, const mpcd_step_args *a, mpcd_best *best_host, float *u_best_host, void *stream)
{
    if (!c || !a || !a->sys || !a->x0 || !a->act_min || !a->act_max || !a->cost_local || !best_host || !u_best_host)
        return fail(MPCD_EINVAL, "null argument");
    if (!c->net_loaded) return fail(MPCD_ESTATE, "no net loaded");
    const mpcd_net_desc &d = c->desc;
    const mpcd_system_desc &sys = *a->sys;
    const int64_t B = a->sample.batch;
    const int H = d.horizon, row = H * d.state_dim;
    if (B < 1 || !a->sample.x_out) return fail(MPCD_EINVAL, "sample.batch / sample.x_out");
    if (sys.n_u != d.state_dim) return fail(MPCD_EINVAL, "system n_u %d != net state_dim %d", sys.n_u, d.state_dim);
    int rc = check_system(&sys, H);
    if (rc) return rc;
    if (d.context_dim > 0 && (!a->ctx_min || !a->ctx_max)) return fail(MPCD_EINVAL, "ctx_min / ctx_max");
    if (d.context_dim > 0 && d.context_dim != sys.n_x) return fail(MPCD_EINVAL, "context_dim %d != n_x %d", d.context_dim, sys.n_x);
    if (c->comm && !a->costs_all) return fail(MPCD_EINVAL, "costs_all is required with a communicator");
    if (a->clip_rule < MPCD_CLIP_CHAIN || a->clip_rule > MPCD_CLIP_NONE) return fail(MPCD_EINVAL, "clip_rule %d", a->clip_rule);
    hipStream_t st = static_cast<hipStream_t>(stream);
    DEVICE_GUARD(c->device);

    // host staging (pinned): [context row | result block]
    // result block: {best, winner row [row] fp32, clip code int32} - one D2H copy
    const size_t out_bytes = sizeof(mpcd_best) + sizeof(float) * (size_t)row + sizeof(int32_t);
    const size_t flag_off = 64 + ((out_bytes + 63) & ~(size_t)63);  // the completion word, own 64-byte line
    const size_t host_bytes = flag_off + 64;
    if (c->step_host_bytes < host_bytes) {
        if (c->step_host) (void)hipHostFree(c->step_host);
        c->step_host = nullptr;
        c->step_host_dev = nullptr;
        c->step_host_bytes = 0;
        // coherent (fine-grained) mapped memory: the selecting workgroup's system-scope stores of the result block
        // and the completion word reach the host without depending on HIP_HOST_COHERENT's default
        HIP_TRY(hipHostMalloc(&c->step_host, host_bytes, hipHostMallocMapped | hipHostMallocCoherent));
        HIP_TRY(hipHostGetDevicePointer(&c->step_host_dev, c->step_host, 0));
        memset(c->step_host, 0, host_bytes);
        c->step_seq = 0;
        c->step_host_bytes = host_bytes;
    }
    if ((rc = c->step_ctx.ensure(64)) || (rc = c->step_out.ensure(out_bytes))) return rc;
    const int64_t n_part = (B + kRolloutBlock - 1) / kRolloutBlock;
    if ((rc = c->step_part.ensure(16 * (size_t)n_part + sizeof(float) * (size_t)row))) return rc;

    // normalize_condition (A12), fp64 then the net's .float()
    mpcd_sample_args sa = a->sample;
    CtxRowArg ctx_row{};
    const bool by_value = d.context_dim > 0 && d.context_dim <= kCtxRowMax;
    if (d.context_dim > 0) {
        float *ch = by_value ? ctx_row.v : static_cast<float *>(c->step_host);
        for (int i = 0; i < d.context_dim; ++i) {
            const double den = (double)(a->ctx_max[i] - a->ctx_min[i]);
            ch[i] = (float)(2.0 * ((a->x0[i] - (double)a->ctx_min[i]) / den) - 1.0);
        }
        if (!by_value)
            HIP_TRY(hipMemcpyAsync(c->step_ctx.p, ch, sizeof(float) * d.context_dim, hipMemcpyHostToDevice, st));
        sa.context = by_value ? nullptr : c->step_ctx.as<float>();
        sa.context_shared = 1;
    } else {
        sa.context = nullptr;
    }
    sa.chain_absmax = nullptr;
    if (a->clip_rule == MPCD_CLIP_CHAIN) {
        if ((rc = c->step_amax.ensure(sizeof(float) * (size_t)B))) return rc;
        sa.chain_absmax = c->step_amax.as<float>();
    }
    if ((rc = sample_impl(c, &sa, stream, by_value ? &ctx_row : nullptr))) return rc;

    // LimitsNormalizer's global clip flag over the chain (the reference's unnormalize_states of run_CFG's
    // whole chain), over the final samples, or proven 0; max-reduced over ranks (see mpcd_clip_flag)
    int *flags = c->flag.as<int>();
    const int *flag = flags + 1;  // flag[1] is never written: a constant 0
    // single rank, a small clip input: the selecting rollout launch computes the clip code itself (each
    // workgroup over the whole input, <= kFuseClipMax floats) - one launch fewer per control step
    const float *clip_src = a->clip_rule == MPCD_CLIP_CHAIN ? sa.chain_absmax : sa.x_out;
    const int64_t clip_n = a->clip_rule == MPCD_CLIP_CHAIN ? B : B * row;
    const bool fuse_clip = !c->comm && a->clip_rule != MPCD_CLIP_NONE && clip_n <= kFuseClipMax;
    if (a->clip_rule != MPCD_CLIP_NONE && !fuse_clip) {
        if (a->clip_rule == MPCD_CLIP_CHAIN)
            HIP_TRY(launch_clip_flag(sa.chain_absmax, B, flags, c->sync_ws(), st));
        else
            HIP_TRY(launch_clip_flag(sa.x_out, B * row, flags, c->sync_ws(), st));
        if ((rc = comm_reduce(c, flags, 1, COMM_MAX_I32, st))) return rc;
        flag = flags;
    }
    mpcd_best *best_dev = c->step_out.as<mpcd_best>();
    float *u_dev = reinterpret_cast<float *>(best_dev + 1);
    double *part_cost = c->step_part.as<double>();
    int64_t *part_idx = reinterpret_cast<int64_t *>(part_cost + n_part);
    int32_t *code_dev = reinterpret_cast<int32_t *>(u_dev + row);
    void *host_out = static_cast<char *>(c->step_host) + 64;
    volatile uint32_t *host_flag = reinterpret_cast<volatile uint32_t *>(static_cast<char *>(c->step_host) + flag_off);
    uint32_t seq = 0;
    if (!c->comm) {  // rollout + cost + argmin + the winner's unnormalised row + the clip code in one launch
        seq = ++c->step_seq;
        if (seq == 0) seq = ++c->step_seq;
        char *hdev = static_cast<char *>(c->step_host_dev);
        RolloutSelect sel{best_dev, u_dev,    part_cost, part_idx, c->sync_ws() + 8, n_part, sa.global_offset, code_dev,
                          fuse_clip ? clip_src : nullptr, fuse_clip ? clip_n : 0, hdev + 64,
                          reinterpret_cast<uint32_t *>(hdev + flag_off), seq};
        HIP_TRY(launch_rollout_cost(sys, a->x0, nullptr, B, sa.x_out, a->act_min, a->act_max, flag, B, H,
                                    a->cost_local, st, &sel));
    } else {
        HIP_TRY(launch_rollout_cost(sys, a->x0, nullptr, B, sa.x_out, a->act_min, a->act_max, flag, B, H,
                                    a->cost_local, st));
        float *row_norm = reinterpret_cast<float *>(part_idx + n_part);
        if ((rc = comm_gather(c, a->cost_local, a->costs_all, (size_t)B, 8, st))) return rc;
        HIP_TRY(launch_argmin(a->costs_all, B * c->nranks, 0, best_dev, st));
        HIP_TRY(launch_winner_row(best_dev, (int64_t)c->rank * B, B, sa.x_out, row, row_norm, st));
        if ((rc = comm_reduce(c, row_norm, (size_t)row, COMM_SUM_F32, st))) return rc;
        HIP_TRY(launch_unnormalize(row_norm, row, d.state_dim, flag, a->act_min, a->act_max, u_dev, st));
        HIP_TRY(hipMemcpyAsync(code_dev, flag, sizeof(int32_t), hipMemcpyDeviceToDevice, st));
    }
    if (c->comm) {
        HIP_TRY(hipMemcpyAsync(host_out, c->step_out.p, out_bytes, hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
    } else {
        // the selecting workgroup wrote the block to mapped host memory and then the completion word: spin on it
        // (no copy launch, no stream synchronisation wake-up); the stream is queried now and then so that a failed
        // launch cannot leave this loop waiting
        for (uint32_t n = 1; *host_flag != seq; ++n) {
            if ((n & 4095) == 0) {
                const hipError_t q = hipStreamQuery(st);
                if (q == hipSuccess && *host_flag != seq)
                    return fail(MPCD_EHIP, "mpcd_mpc_step: the stream finished without the result block");
                if (q != hipSuccess && q != hipErrorNotReady) HIP_TRY(q);
            }
#if defined(__x86_64__) || defined(__i386__)
            __builtin_ia32_pause();  // spin-wait hint (host CPU)
#else
            std::this_thread::yield();
#endif
        }
        std::atomic_thread_fence(std::memory_order_acquire);
    }
    memcpy(best_host, host_out, sizeof(mpcd_best));
    memcpy(u_best_host, static_cast<char *>(host_out) + sizeof(mpcd_best), sizeof(float) * (size_t)row);
    int32_t code = 0;
    memcpy(&code, static_cast<char *>(host_out) + sizeof(mpcd_best) + sizeof(float) * (size_t)row, sizeof code);
    c->step_flags = (code == 1 ? MPCD_STEP_CLIPPED : 0) | (code == 2 ? MPCD_STEP_NAN_SAMPLES : 0);
    if (!std::isfinite(best_host->cost)) {
        c->step_flags |= MPCD_STEP_NONFINITE_WINNER;
        return fail(MPCD_ENONFINITE, "mpcd_mpc_step: no candidate has a finite cost (best %g, index %lld)%s",
                    best_host->cost, (long long)best_host->index,
                    code == 2 ? "; NaN in the sampled trajectories" : "");
    }
    return MPCD_OK;
}


// ---- native training step: MLP noise-net, fp32, csrc/train.hip

struct mpcd_trainer {
    Trainer *t = nullptr;
    int64_t n_params = 0;
    int device = 0;  // the device current at mpcd_trainer_create: owns every buffer; each call switches to it
};

int mpcd_trainer_create(const mpcd_net_desc *desc, const float *params, size_t n_floats, const mpcd_train_cfg *cfg,
                        const float *sqrt_alphas_cumprod, const float *sqrt_one_minus_alphas_cumprod, int32_t n_steps,
                        mpcd_trainer **out)
{
    if (!out) return fail(MPCD_EINVAL, "null out");
    *out = nullptr;
    if (int r = check_desc(desc)) return r;
    if (desc->kind == MPCD_NET_UNET && !desc->cfg_masked)
        return fail(MPCD_EUNSUP, "mpcd_trainer: the 3-arg TemporalUnet is not trainable here (ConditionedTemporalUnet is)");
    if (!params || !cfg || !sqrt_alphas_cumprod || !sqrt_one_minus_alphas_cumprod || n_steps < 1)
        return fail(MPCD_EINVAL, "mpcd_trainer_create: null argument or no schedule");
    const std::vector<PSpec> spec = param_spec(*desc);
    std::map<std::string, int64_t> off;
    int64_t o = 0;
    for (const PSpec &p : spec) {
        off[p.name] = o;
        o += p.numel();
    }
    if ((size_t)o != n_floats) return fail(MPCD_EINVAL, "mpcd_trainer_create: %zu floats, the net has %lld", n_floats, (long long)o);
    auto lin = [&](const std::string &pre, int n, int k) {
        TrainLin L;
        L.w = off.at(pre + ".weight");
        L.b = off.at(pre + ".bias");
        L.n = n;
        L.k = k;
        return L;
    };
    TrainSpec sp;
    sp.flat = desc->horizon * desc->state_dim;
    sp.temb = desc->time_emb_dim;
    sp.ctx_dim = desc->context_dim;
    sp.base = desc->base_dim;
    sp.n_steps = n_steps;
    sp.n_params = o;
    sp.lr = cfg->lr;
    sp.beta1 = cfg->beta1;
    sp.beta2 = cfg->beta2;
    sp.eps = cfg->eps;
    sp.ema_decay = cfg->ema_decay;
    sp.step_start_ema = cfg->step_start_ema;
    sp.update_ema_every = cfg->update_ema_every;
    const int cond = cond_dim_of(*desc);
    sp.t1 = lin("time_mlp.encoder.1", 128, 32);
    sp.t2 = lin("time_mlp.encoder.3", desc->time_emb_dim, 128);
    if (desc->kind == MPCD_NET_UNET) {  // ConditionedTemporalUnet trunk (temporal_unet.py:317-358) as an op tape
        sp.unet = true;
        const int H = desc->horizon, d = desc->state_dim, W = cond;
        for (int i = 0; i + 1 < desc->n_mults; ++i)
            if ((H >> (i + 1)) << (i + 1) != H) return fail(MPCD_EINVAL, "mpcd_trainer: horizon %d does not halve %d times", H, desc->n_mults - 1);
        sp.ut = {UTensor{H, d}, UTensor{1, W}};
        auto T = [&](int L, int C) {
            sp.ut.push_back(UTensor{L, C});
            return (int)sp.ut.size() - 1;
        };
        auto add_op = [&](int kind, int in0, int in1, int out, const std::string &pre, int k, int s_, int p_, int g) {
            UOp o;
            o.kind = kind;
            o.in0 = in0;
            o.in1 = in1;
            o.out = out;
            if (!pre.empty()) {
                o.w = off.at(pre + ".weight");
                o.b = off.at(pre + ".bias");
            }
            o.k = k;
            o.s = s_;
            o.p = p_;
            o.groups = g;
            sp.uops.push_back(o);
            return out;
        };
        auto ngroups = [](int c) {
            if (c < 8) return 1;
            for (int g = 8; g < 18; ++g)
                if (c % g == 0) return g;
            return 1;
        };
        auto L_ = [&](int t) { return sp.ut[t].L; };
        auto C_ = [&](int t) { return sp.ut[t].C; };
        auto conv = [&](int x0, int x1, int Lo, int co, const std::string &pre, int k, int s_, int p_) {
            return add_op(UOP_CONV, x0, x1, T(Lo, co), pre, k, s_, p_, 1);
        };
        auto gn = [&](int x, const std::string &pre) { return add_op(UOP_GN, x, -1, T(L_(x), C_(x)), pre, 1, 1, 0, ngroups(C_(x))); };
        auto mish = [&](int x) { return add_op(UOP_MISH, x, -1, T(L_(x), C_(x)), "", 1, 1, 0, 1); };
        auto rtb = [&](int x0, int x1, int co, const std::string &pre) {  // ResidualTemporalBlock (layers.py:323-355)
            const int L = L_(x0), cin = C_(x0) + (x1 >= 0 ? C_(x1) : 0);
            const int m1 = mish(gn(conv(x0, x1, L, co, pre + ".blocks.0.block.0", 5, 1, 2), pre + ".blocks.0.block.2"));
            const int cc = add_op(UOP_LIN, UT_MC, -1, T(1, co), pre + ".cond_mlp.1", 1, 1, 0, 1);
            const int h = add_op(UOP_ADDC, m1, cc, T(L, co), "", 1, 1, 0, 1);
            const int m2 = mish(gn(conv(h, -1, L, co, pre + ".blocks.1.block.0", 5, 1, 2), pre + ".blocks.1.block.2"));
            const int r = cin != co ? conv(x0, x1, L, co, pre + ".residual_conv", 1, 1, 0) : x0;
            return add_op(UOP_ADD, m2, r, T(L, co), "", 1, 1, 0, 1);
        };
        auto st = stages(d, *desc);
        const int nres = (int)st.size();
        int x = UT_XNOISY;
        std::vector<int> skips;
        for (int i = 0; i < nres; ++i) {
            const std::string p = "downs." + std::to_string(i);
            x = rtb(x, -1, st[i].second, p + ".0");
            x = rtb(x, -1, st[i].second, p + ".1");
            skips.push_back(x);
            if (i < nres - 1) x = conv(x, -1, L_(x) / 2, st[i].second, p + ".4.conv", 3, 2, 1);
        }
        x = rtb(x, -1, st.back().second, "mid_block1");
        x = rtb(x, -1, st.back().second, "mid_block2");
        for (int i = 1; i < nres; ++i) {
            const int ci = st[nres - i].first;
            const std::string p = "ups." + std::to_string(i - 1);
            const int skip = skips.back();
            skips.pop_back();
            x = rtb(x, skip, ci, p + ".0");
            x = rtb(x, -1, ci, p + ".1");
            x = add_op(UOP_CONVT, x, -1, T(2 * L_(x), ci), p + ".4.conv", 4, 2, 1, 1);
        }
        x = mish(gn(conv(x, -1, H, desc->base_dim, "final_conv.0.block.0", 5, 1, 2), "final_conv.0.block.2"));
        sp.u_out = add_op(UOP_LIN, x, -1, T(H, d), "final_conv.1", 1, 1, 0, 1);
        if (L_(sp.u_out) != H) return fail(MPCD_EINVAL, "mpcd_trainer: U-Net tape ends at %d positions, not %d", L_(sp.u_out), H);
        (void)W;
    }
    auto st = stages(sp.flat, *desc);
    const int ns = (int)st.size();
    auto block = [&](const std::string &p, int ci, int co, int in0, int in1) {
        TrainBlock b;
        b.la = lin(p + ".blocks.0._network.0", co, ci);
        b.lb = lin(p + ".blocks.0._network.2", co, co);
        b.lc = lin(p + ".cond_mlp.1", co, cond);
        b.co = co;
        b.in0 = in0;
        b.in1 = in1;
        return b;
    };
    for (int i = 0; i < ns && !sp.unet; ++i)
        sp.blocks.push_back(block("downs." + std::to_string(i) + ".0", st[i].first, st[i].second, i - 1, -1));
    if (!sp.unet) sp.blocks.push_back(block("mid_block1", st.back().second, st.back().second, ns - 1, -1));
    for (int i = 1; i < ns && !sp.unet; ++i) {  // ups.{i-1}: cat(previous output, skip = downs.{ns-i})
        auto [ci, co] = st[ns - i];
        sp.blocks.push_back(block("ups." + std::to_string(i - 1) + ".0", 2 * co, ci, (int)sp.blocks.size() - 1, ns - i));
    }
    if (!sp.unet) {
        sp.f1 = lin("final_layer.0._network.0", desc->base_dim, desc->base_dim);
        sp.f2 = lin("final_layer.0._network.2", sp.flat, desc->base_dim);
    }
    std::vector<float> sched((size_t)2 * n_steps);
    std::copy(sqrt_alphas_cumprod, sqrt_alphas_cumprod + n_steps, sched.begin());
    std::copy(sqrt_one_minus_alphas_cumprod, sqrt_one_minus_alphas_cumprod + n_steps, sched.begin() + n_steps);
    std::string why;
    int dev = 0;
    HIP_TRY(hipGetDevice(&dev));
    Trainer *t = trainer_new(sp, params, sched.data(), &why);
    if (!t) return fail(MPCD_ENOMEM, "%s", why.c_str());
    *out = new mpcd_trainer{t, o, dev};
    return MPCD_OK;
}

int mpcd_trainer_step(mpcd_trainer *tr, const float *x0, const float *context, const int64_t *t, const float *noise,
                      const float *context_mask, int64_t batch, int32_t update, double *loss, void *hip_stream)
{
    if (!tr || !x0 || !context || !t || !noise || !context_mask || !loss || batch < 1)
        return fail(MPCD_EINVAL, "mpcd_trainer_step: null argument or empty batch");
    DEVICE_GUARD(tr->device);
    TrainBatch b{x0, context, noise, context_mask, t, batch, hip_stream};
    std::string why;
    const int r = trainer_step(tr->t, b, update != 0, loss, &why);
    if (r == -1) return fail(MPCD_ENOMEM, "%s", why.c_str());
    if (r != 0) return fail(MPCD_EHIP, "%s", why.c_str());
    return MPCD_OK;
}

int mpcd_trainer_params(mpcd_trainer *tr, int32_t which, float *host_out, size_t n_floats)
{
    if (!tr || !host_out || which < 0 || which > 4) return fail(MPCD_EINVAL, "mpcd_trainer_params: bad argument");
    DEVICE_GUARD(tr->device);
    const int r = trainer_read(tr->t, which, host_out, n_floats);
    if (r == -1) return fail(MPCD_EINVAL, "mpcd_trainer_params: %zu floats, the net has %lld", n_floats, (long long)tr->n_params);
    if (r != 0) return fail(MPCD_EHIP, "mpcd_trainer_params: copy failed");
    return MPCD_OK;
}

int mpcd_trainer_comm_init(mpcd_trainer *tr, int32_t nranks, int32_t rank, const void *id_in)
{
    if (!tr || !id_in || nranks < 1 || rank < 0 || rank >= nranks) return fail(MPCD_EINVAL, "bad comm arguments");
    DEVICE_GUARD(tr->device);
    std::string e;
    Comm *c = nullptr;
    if (int rc = comm_create_rccl(nranks, rank, id_in, &c, e)) return fail(rc, "%s", e.c_str());
    if (trainer_set_comm(tr->t, c)) {
        delete c;
        return fail(MPCD_ESTATE, "trainer communicator already initialised");
    }
    return MPCD_OK;
}

int mpcd_trainer_comm_init_loopback(mpcd_trainer *tr, int32_t nranks, int32_t rank, uint64_t group_key)
{
    if (!tr || nranks < 1 || rank < 0 || rank >= nranks) return fail(MPCD_EINVAL, "bad comm arguments");
    DEVICE_GUARD(tr->device);
    std::string e;
    Comm *c = nullptr;
    if (int rc = comm_create_loopback(nranks, rank, group_key, &c, e)) return fail(rc, "%s", e.c_str());
    if (trainer_set_comm(tr->t, c)) {
        delete c;
        return fail(MPCD_ESTATE, "trainer communicator already initialised");
    }
    return MPCD_OK;
}

void mpcd_trainer_destroy(mpcd_trainer *tr)
{
    if (!tr) return;
    DeviceGuard device_guard_(tr->device);
    trainer_free(tr->t);
    delete tr;
}

}  // extern "C"
