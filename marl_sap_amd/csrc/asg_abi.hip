// asg_abi.hip -- the extern "C" boundary (include/asg.h): handle lifecycle, argument
// validation, error strings, and dispatch to the kernels.  No exception crosses it.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <new>
#include <string>

#include "../../include/asg.h"
#include "asg_internal.h"

using asg::EnvState;

struct asg_handle {
    EnvState st{};
    hipStream_t stream = nullptr;
    int device = 0;
    int k = 0;                 // steps taken in the current episode
    bool has_reset = false;
    bool constructed = false;  // MT19937: first reset also replays __init__'s draw
    bool table_ready = false;  // injected table uploaded
    // bids_as_actions: the bids row whose LSA assignments st.assign holds (asg_bids_select wrote
    // both); a step on that row uses them instead of solving the row again.  Cleared by resets.
    struct BidsTag {
        const float *row = nullptr;
        int64_t s_env = 0, s_agent = 0, s_task = 0;
    } bids_tag;
    std::string err;
};

namespace {

thread_local std::string g_err;

int fail(asg_handle *h, int code, const std::string &msg) {
    g_err = msg;
    if (h) h->err = msg;
    return code;
}

int hip_fail(asg_handle *h, hipError_t e, const char *what) {
    return fail(h, ASG_E_HIP, std::string(what) + ": " + hipGetErrorString(e));
}

// keeps the caller's current device (PyTorch tracks its own) around every entry point
struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != dev) (void)hipSetDevice(dev);
    }
    ~DeviceGuard() {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
};

bool field_ok(const asg_field &f, int want_dtype) { return f.ptr == nullptr || f.dtype == want_dtype; }

int check_view(asg_handle *h, const asg_batch_view *b, int ts, bool step) {
    if (!b) return fail(h, ASG_E_INVALID_ARG, "batch view is NULL");
    const EnvState &st = h->st;
    if (ts < 0 || (step && ts + 1 > st.T + 64 * 1024)) return fail(h, ASG_E_INVALID_ARG, "bad ts");
    if (!b->obs.ptr) return fail(h, ASG_E_INVALID_ARG, "obs field is required");
    if (!field_ok(b->obs, ASG_F32) || !field_ok(b->beta, ASG_F32) || !field_ok(b->rewards, ASG_F32) ||
        !field_ok(b->avail_actions, ASG_BOOL) || !field_ok(b->terminated, ASG_BOOL) ||
        !field_ok(b->prev_assigns, ASG_I64) || !field_ok(b->actions_onehot, ASG_I64) ||
        !field_ok(b->filled, ASG_I64))
        return fail(h, ASG_E_INVALID_ARG, "batch field dtype does not match the env scheme");
    if (step) {
        if (!b->actions.ptr) return fail(h, ASG_E_INVALID_ARG, "actions field is required for step");
        if (!field_ok(b->actions, st.bids ? ASG_F32 : ASG_I64))
            return fail(h, ASG_E_INVALID_ARG,
                        st.bids ? "bids_as_actions expects float32 actions" : "actions must be int64");
    }
    return ASG_OK;
}

// bids_as_actions: does st.assign hold the assignments of batch row ts (asg_bids_select)?
bool bids_ready(const asg_handle *h, const asg_batch_view *b, int ts) {
    const asg_field &f = b->actions;
    const float *row = static_cast<const float *>(f.ptr) + (int64_t)ts * f.stride[1];
    const auto &t = h->bids_tag;
    return h->st.bids && t.row && t.row == row && t.s_env == f.stride[0] && t.s_agent == f.stride[2] &&
           t.s_task == f.stride[3];
}

// ASG_STEP_USE_SELECTED_BIDS: the caller states that batch row ts still holds the bids
// asg_bids_select wrote (nothing wrote the row since); the handle checks that it is that row.
// Without the flag every step solves the row it is given.
int selected_bids_ok(asg_handle *h, const asg_batch_view *b, int ts, int flags) {
    if (!(flags & ASG_STEP_USE_SELECTED_BIDS)) return ASG_OK;
    if (!h->st.bids) return fail(h, ASG_E_INVALID_ARG, "ASG_STEP_USE_SELECTED_BIDS needs a bids_as_actions handle");
    if (!bids_ready(h, b, ts))
        return fail(h, ASG_E_STATE,
                    "ASG_STEP_USE_SELECTED_BIDS: batch row ts is not the row asg_bids_select last wrote "
                    "(or a step / reset came in between)");
    return ASG_OK;
}

}  // namespace

void asg::set_last_error(const std::string &msg) { g_err = msg; }

extern "C" {

int asg_abi_version(void) { return ASG_ABI_VERSION; }

const char *asg_last_error(const asg_handle *h) { return h ? h->err.c_str() : g_err.c_str(); }

int asg_create(const asg_config *cfg, int device, void *hip_stream, asg_handle **out) {
    if (!cfg || !out) return fail(nullptr, ASG_E_INVALID_ARG, "cfg and out must be non-NULL");
    *out = nullptr;
    if (cfg->num_envs <= 0 || cfg->n <= 0 || cfg->m <= 0 || cfg->T <= 0 || cfg->L < 0)
        return fail(nullptr, ASG_E_INVALID_ARG, "num_envs, n, m, T must be positive and L >= 0");
    if (cfg->n > cfg->m)
        return fail(nullptr, ASG_E_INVALID_ARG,
                    "Cannot take a larger sample than population when 'replace=False' (reset draws "
                    "choice(m, n, replace=False): needs n <= m)");
    if (cfg->n > 4096 || cfg->m > 1024)
        return fail(nullptr, ASG_E_INVALID_ARG, "n <= 4096 and m <= 1024 are supported");
    if (cfg->rng_mode != ASG_RNG_PHILOX && cfg->rng_mode != ASG_RNG_MT19937)
        return fail(nullptr, ASG_E_INVALID_ARG, "unknown rng_mode");
    if (cfg->benefit_mode < ASG_BENEFIT_BUMP || cfg->benefit_mode > ASG_BENEFIT_INJECTED)
        return fail(nullptr, ASG_E_INVALID_ARG, "unknown benefit_mode");
    if (cfg->bids_as_actions && (int64_t)cfg->n * cfg->m > 16384)
        return fail(nullptr, ASG_E_INVALID_ARG, "bids_as_actions supports n * m <= 16384 (the bid matrix is solved in LDS)");
    if (cfg->rng_mode == ASG_RNG_MT19937 && cfg->benefit_mode == ASG_BENEFIT_DENSE)
        return fail(nullptr, ASG_E_INVALID_ARG, "dense benefits are a Philox-mode workload");
    asg_handle *h = new (std::nothrow) asg_handle();
    if (!h) return fail(nullptr, ASG_E_HIP, "out of host memory");
    DeviceGuard g(device);
    h->device = device;
    h->stream = static_cast<hipStream_t>(hip_stream);
    EnvState &st = h->st;
    st.E = cfg->num_envs;
    st.n = cfg->n;
    st.m = cfg->m;
    st.T = cfg->T;
    st.L = cfg->L;
    st.lambda_ = cfg->lambda_;
    st.bids = cfg->bids_as_actions ? 1 : 0;
    st.rng_mode = cfg->rng_mode;
    st.benefit_mode = cfg->benefit_mode;
    st.quirks = cfg->quirks;
    st.seed = cfg->seed;
    st.env_base = cfg->env_index_base;
    st.episode = 0;
    st.wmin_init = 5.0;
    st.wmax_init = 8.0;
    st.wmin = 3.0;
    st.wmax = 6.0;
    const size_t E = (size_t)st.E, n = st.n, m = st.m, T = st.T;
    hipError_t e;
    if ((e = hipMalloc(&st.prev, sizeof(int) * E * n)) != hipSuccess) goto oom;
    if ((e = hipMalloc(&st.returns, sizeof(double) * E)) != hipSuccess) goto oom;
    if ((e = hipMalloc(&st.err, sizeof(int))) != hipSuccess) goto oom;
    if ((e = hipMemsetAsync(st.err, 0, sizeof(int), h->stream)) != hipSuccess) goto oom;
    if ((e = hipMemsetAsync(st.returns, 0, sizeof(double) * E, h->stream)) != hipSuccess) goto oom;
    if ((e = hipMemsetAsync(st.prev, 0, sizeof(int) * E * n, h->stream)) != hipSuccess) goto oom;
    if (cfg->T_trans) {
        double *tt = nullptr;
        if ((e = hipMalloc(&tt, sizeof(double) * m * m)) != hipSuccess) goto oom;
        if ((e = hipMemcpy(tt, cfg->T_trans, sizeof(double) * m * m, hipMemcpyHostToDevice)) != hipSuccess) goto oom;
        st.T_trans = tt;
    }
    if (st.benefit_mode == ASG_BENEFIT_INJECTED) {
        if ((e = hipMalloc(&st.table, sizeof(double) * E * T * n * m)) != hipSuccess) goto oom;
        if ((e = hipMemsetAsync(st.table, 0, sizeof(double) * E * T * n * m, h->stream)) != hipSuccess) goto oom;
    }
    if (st.rng_mode == ASG_RNG_MT19937 || st.benefit_mode == ASG_BENEFIT_INJECTED) {
        // + 16 floats: the compact table's 16-byte quad reads may run 12 bytes past a slice's pairs
        if ((e = hipMalloc(&st.table32, sizeof(float) * (E * T * n * m + 16))) != hipSuccess) goto oom;
        if ((e = hipMemsetAsync(st.table32, 0, sizeof(float) * (E * T * n * m + 16), h->stream)) != hipSuccess) goto oom;
    }
    if (st.rng_mode == ASG_RNG_MT19937 && st.benefit_mode != ASG_BENEFIT_INJECTED) {
        // the compact table's pair masks / offsets (all zero = no bumps, the zero table before a reset)
        const size_t W = (m + 63) / 64;
        if ((e = hipMalloc(&st.tmask, sizeof(uint64_t) * E * n * W)) != hipSuccess) goto oom;
        if ((e = hipMemsetAsync(st.tmask, 0, sizeof(uint64_t) * E * n * W, h->stream)) != hipSuccess) goto oom;
        if ((e = hipMalloc(&st.toff, sizeof(int) * E * n * W)) != hipSuccess) goto oom;
        if ((e = hipMemsetAsync(st.toff, 0, sizeof(int) * E * n * W, h->stream)) != hipSuccess) goto oom;
    }
    if (st.bids) {
        if ((e = hipMalloc(&st.assign, sizeof(int) * E * n)) != hipSuccess) goto oom;
    }
    if (st.rng_mode == ASG_RNG_MT19937) {
        if ((e = hipMalloc(&st.mt, sizeof(uint32_t) * E * 625)) != hipSuccess) goto oom;
        if (st.benefit_mode != ASG_BENEFIT_INJECTED) {  // zero draws = the zero table before a reset
            if ((e = hipMalloc(&st.mtpar, sizeof(double2) * E * n * m)) != hipSuccess) goto oom;
            if ((e = hipMemsetAsync(st.mtpar, 0, sizeof(double2) * E * n * m, h->stream)) != hipSuccess) goto oom;
        }
        if ((e = asg::launch_mt_seed(st, h->stream)) != hipSuccess) goto oom;
    }
    *out = h;
    return ASG_OK;
oom:
    {
        const int rc = hip_fail(nullptr, e, "asg_create");
        asg_destroy(h);
        return rc;
    }
}

int asg_destroy(asg_handle *h) {
    if (!h) return ASG_OK;
    DeviceGuard g(h->device);
    if (h->stream) (void)hipStreamSynchronize(h->stream);
    else (void)hipDeviceSynchronize();
    EnvState &st = h->st;
    (void)hipFree(st.prev);
    (void)hipFree(st.returns);
    (void)hipFree(st.err);
    (void)hipFree(const_cast<double *>(st.T_trans));
    (void)hipFree(st.table);
    (void)hipFree(st.table32);
    (void)hipFree(st.tmask);
    (void)hipFree(st.toff);
    (void)hipFree(st.mt);
    (void)hipFree(st.mtpar);
    (void)hipFree(st.assign);
    delete h;
    return ASG_OK;
}

int asg_set_stream(asg_handle *h, void *hip_stream) {
    if (!h) return fail(nullptr, ASG_E_INVALID_ARG, "NULL handle");
    h->stream = static_cast<hipStream_t>(hip_stream);
    return ASG_OK;
}

int asg_reset(asg_handle *h, const asg_batch_view *b, int ts) {
    if (!h) return fail(nullptr, ASG_E_INVALID_ARG, "NULL handle");
    if (int rc = check_view(h, b, ts, false)) return rc;
    if (h->st.benefit_mode == ASG_BENEFIT_INJECTED && !h->table_ready)
        return fail(h, ASG_E_STATE, "benefit_mode=injected needs asg_set_benefits before reset");
    DeviceGuard g(h->device);
    // Philox: a fresh key per episode (first = 0), committed to the handle only once the
    // launch succeeded (a failed launch leaves the handle as it was)
    asg::EnvState st = h->st;
    if (h->has_reset) st.episode += 1;
    hipError_t e = asg::launch_reset(*b, st, ts, !h->constructed, h->stream);
    if (e != hipSuccess) return hip_fail(h, e, "asg_reset");
    h->st.episode = st.episode;
    h->constructed = true;
    h->has_reset = true;
    h->k = 0;
    h->bids_tag = {};
    return ASG_OK;
}

int asg_step(asg_handle *h, const asg_batch_view *b, int ts) { return asg_step_ex(h, b, ts, 0); }

int asg_step_ex(asg_handle *h, const asg_batch_view *b, int ts, int flags) {
    if (!h) return fail(nullptr, ASG_E_INVALID_ARG, "NULL handle");
    if (int rc = check_view(h, b, ts, true)) return rc;
    if (!h->has_reset) return fail(h, ASG_E_STATE, "step called before reset");
    if (h->k >= h->st.T) return fail(h, ASG_E_STATE, "episode already terminated (k >= T); reset first");
    if (flags & ~ASG_STEP_USE_SELECTED_BIDS) return fail(h, ASG_E_INVALID_ARG, "asg_step_ex: unknown flags");
    if (int rc = selected_bids_ok(h, b, ts, flags)) return rc;
    DeviceGuard g(h->device);
    const bool ready = (flags & ASG_STEP_USE_SELECTED_BIDS) != 0;
    hipError_t e = asg::launch_step(*b, h->st, ts, h->k, h->stream, ready);
    if (e != hipSuccess) return hip_fail(h, e, "asg_step");
    h->k += 1;
    h->bids_tag = {};
    return ASG_OK;
}

int asg_random_actions(asg_handle *h, const asg_batch_view *b, int ts) {
    if (!h) return fail(nullptr, ASG_E_INVALID_ARG, "NULL handle");
    if (!b || !b->actions.ptr || b->actions.dtype != ASG_I64)
        return fail(h, ASG_E_INVALID_ARG, "random actions need an int64 actions field");
    DeviceGuard g(h->device);
    hipError_t e = asg::launch_random_actions(*b, h->st, ts, h->k, h->stream);
    if (e != hipSuccess) return hip_fail(h, e, "asg_random_actions");
    return ASG_OK;
}

int asg_random_rollout(asg_handle *h, const asg_batch_view *b, int ts, int steps, int reset) {
    if (!h) return fail(nullptr, ASG_E_INVALID_ARG, "NULL handle");
    if (int rc = check_view(h, b, ts, false)) return rc;
    const asg::EnvState &st = h->st;
    if (st.bids) return fail(h, ASG_E_INVALID_ARG, "asg_random_rollout: integer actions only (not bids_as_actions)");
    if (b->actions.ptr && b->actions.dtype != ASG_I64)
        return fail(h, ASG_E_INVALID_ARG, "random actions need an int64 actions field");
    if (reset && st.rng_mode == ASG_RNG_MT19937)
        return fail(h, ASG_E_INVALID_ARG, "asg_random_rollout: the MT19937 mode's reset is asg_reset (its stream)");
    if (reset && st.benefit_mode == ASG_BENEFIT_INJECTED && !h->table_ready)
        return fail(h, ASG_E_STATE, "benefit_mode=injected needs asg_set_benefits before reset");
    if (!h->has_reset && !reset) return fail(h, ASG_E_STATE, "step called before reset");
    const int k0 = reset ? 0 : h->k;
    if (steps < 1 || k0 + steps > st.T)
        return fail(h, ASG_E_STATE, "asg_random_rollout: steps must be >= 1 and stay within the episode (k + steps <= T)");
    if (ts < 0 || ts + steps > st.T)
        return fail(h, ASG_E_INVALID_ARG, "asg_random_rollout: batch rows ts .. ts + steps must lie in the [T + 1]-row batch");
    DeviceGuard g(h->device);
    asg::EnvState lst = h->st;
    if (reset && h->has_reset) lst.episode += 1;  // as asg_reset: a fresh Philox key per episode
    hipError_t e = asg::launch_random_rollout(*b, lst, ts, k0, steps, reset != 0, h->stream);
    if (e != hipSuccess) return hip_fail(h, e, "asg_random_rollout");
    h->st.episode = lst.episode;
    if (reset) {
        h->constructed = true;
        h->has_reset = true;
    }
    h->k = k0 + steps;
    return ASG_OK;
}

int asg_sync_status(asg_handle *h) {
    if (!h) return fail(nullptr, ASG_E_INVALID_ARG, "NULL handle");
    DeviceGuard g(h->device);
    int code = 0;
    hipError_t e = hipMemcpyAsync(&code, h->st.err, sizeof(int), hipMemcpyDeviceToHost, h->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
    if (e != hipSuccess) return hip_fail(h, e, "asg_sync_status");
    if (code != 0) {
        (void)hipMemsetAsync(h->st.err, 0, sizeof(int), h->stream);
        if (code == ASG_E_ACTION_RANGE)
            return fail(h, code, "an action outside [0, m) was passed to step (OneHot / task index out of range)");
        if (code == ASG_E_LSA_INVALID) return fail(h, code, "matrix contains invalid numeric entries");
        if (code == ASG_E_LSA_INFEASIBLE) return fail(h, code, "cost matrix is infeasible");
        return fail(h, code, "device error " + std::to_string(code));
    }
    return ASG_OK;
}

int asg_set_benefits(asg_handle *h, const double *table, int64_t count, int on_device) {
    if (!h) return fail(nullptr, ASG_E_INVALID_ARG, "NULL handle");
    EnvState &st = h->st;
    const int64_t per = (int64_t)st.n * st.m * st.T;
    if (!table || (count != per && count != per * st.E))
        return fail(h, ASG_E_INVALID_ARG, "benefit table must hold n*m*T (broadcast) or E*n*m*T doubles");
    if (st.benefit_mode != ASG_BENEFIT_INJECTED)
        return fail(h, ASG_E_STATE, "handle was not created with benefit_mode=injected");
    DeviceGuard g(h->device);
    const double *src = table;
    double *tmp = nullptr;
    hipError_t e = hipSuccess;
    if (!on_device) {
        if ((e = hipMalloc(&tmp, sizeof(double) * count)) != hipSuccess) return hip_fail(h, e, "asg_set_benefits");
        if ((e = hipMemcpyAsync(tmp, table, sizeof(double) * count, hipMemcpyHostToDevice, h->stream)) != hipSuccess) {
            (void)hipFree(tmp);
            return hip_fail(h, e, "asg_set_benefits");
        }
        src = tmp;
    }
    e = asg::launch_import_table(src, count == per ? 1 : st.E, st, h->stream);
    if (tmp) {
        (void)hipStreamSynchronize(h->stream);
        (void)hipFree(tmp);
    }
    if (e != hipSuccess) return hip_fail(h, e, "asg_set_benefits");
    h->table_ready = true;
    return ASG_OK;
}

int asg_export_benefits(asg_handle *h, double *out_dev) {
    if (!h || !out_dev) return fail(h, ASG_E_INVALID_ARG, "NULL argument");
    if (!h->has_reset) return fail(h, ASG_E_STATE, "no episode yet: reset first");
    DeviceGuard g(h->device);
    hipError_t e = asg::launch_export_table(h->st, out_dev, h->stream);
    return e == hipSuccess ? ASG_OK : hip_fail(h, e, "asg_export_benefits");
}

int asg_export_bump_params(asg_handle *h, float *out_dev) {
    if (!h || !out_dev) return fail(h, ASG_E_INVALID_ARG, "NULL argument");
    if (!h->has_reset) return fail(h, ASG_E_STATE, "no episode yet: reset first");
    if (h->st.rng_mode != ASG_RNG_PHILOX || h->st.benefit_mode == ASG_BENEFIT_INJECTED)
        return fail(h, ASG_E_INVALID_ARG, "asg_export_bump_params: only Philox bump / dense benefits have parameters");
    DeviceGuard g(h->device);
    hipError_t e = asg::launch_export_bump_params(h->st, out_dev, h->stream);
    return e == hipSuccess ? ASG_OK : hip_fail(h, e, "asg_export_bump_params");
}

int asg_export_prev_assigns(asg_handle *h, int64_t *out_dev) {
    if (!h || !out_dev) return fail(h, ASG_E_INVALID_ARG, "NULL argument");
    DeviceGuard g(h->device);
    hipError_t e = asg::launch_export_prev(h->st, out_dev, h->stream);
    return e == hipSuccess ? ASG_OK : hip_fail(h, e, "asg_export_prev_assigns");
}

int asg_get_returns(asg_handle *h, double *out_dev) {
    if (!h || !out_dev) return fail(h, ASG_E_INVALID_ARG, "NULL argument");
    DeviceGuard g(h->device);
    hipError_t e = hipMemcpyAsync(out_dev, h->st.returns, sizeof(double) * h->st.E, hipMemcpyDeviceToDevice,
                                  h->stream);
    return e == hipSuccess ? ASG_OK : hip_fail(h, e, "asg_get_returns");
}

int asg_get_step(const asg_handle *h, int *k_out) {
    if (!h || !k_out) return fail(nullptr, ASG_E_INVALID_ARG, "NULL argument");
    *k_out = h->k;
    return ASG_OK;
}

int asg_advance_stream(asg_handle *h, int64_t words) {
    if (!h) return fail(nullptr, ASG_E_INVALID_ARG, "NULL handle");
    if (h->st.rng_mode != ASG_RNG_MT19937) return fail(h, ASG_E_STATE, "only MT19937 streams can be advanced");
    if (words < 0) return fail(h, ASG_E_INVALID_ARG, "words must be >= 0");
    DeviceGuard g(h->device);
    hipError_t e = asg::launch_mt_advance(h->st, words, h->stream);
    return e == hipSuccess ? ASG_OK : hip_fail(h, e, "asg_advance_stream");
}

int asg_beta_hat(const void *beta, int beta_dtype, const int64_t beta_strides[3], const int64_t *prev,
                 const int64_t prev_strides[2], int64_t B, int n, int m, const double *T_trans_dev, double lambda_,
                 double *out, void *hip_stream) {
    if (!beta || !beta_strides || !prev || !prev_strides || !out || B < 0 || n <= 0 || m <= 0)
        return fail(nullptr, ASG_E_INVALID_ARG, "asg_beta_hat: bad arguments");
    if (beta_dtype != ASG_F32 && beta_dtype != ASG_F64)
        return fail(nullptr, ASG_E_INVALID_ARG, "asg_beta_hat: beta must be float32 or float64");
    if (B == 0) return ASG_OK;
    hipError_t e = asg::launch_beta_hat(beta, beta_dtype, beta_strides, prev, prev_strides, B, n, m, T_trans_dev,
                                        lambda_, out, static_cast<hipStream_t>(hip_stream));
    return e == hipSuccess ? ASG_OK : hip_fail(nullptr, e, "asg_beta_hat");
}

int asg_lsa_batched(const void *C, int dtype, const int64_t strides[3], int64_t B, int nr, int nc, int maximize,
                    int64_t *row_out, int64_t *col_out, int32_t *status_out, void *hip_stream) {
    if (B < 0 || nr < 0 || nc < 0 || !strides) return fail(nullptr, ASG_E_INVALID_ARG, "asg_lsa_batched: bad shape");
    if (dtype != ASG_F32 && dtype != ASG_F64)
        return fail(nullptr, ASG_E_INVALID_ARG, "asg_lsa_batched: cost must be float32 or float64");
    if ((nr > nc ? nr : nc) > 1024) return fail(nullptr, ASG_E_INVALID_ARG, "asg_lsa_batched: max(nr, nc) <= 1024");
    if (B == 0 || nr == 0 || nc == 0) return ASG_OK;
    if (!C) return fail(nullptr, ASG_E_INVALID_ARG, "asg_lsa_batched: NULL cost");
    hipError_t e = asg::launch_lsa_batched(C, dtype, strides, B, nr, nc, maximize, row_out, col_out, status_out,
                                           static_cast<hipStream_t>(hip_stream));
    return e == hipSuccess ? ASG_OK : hip_fail(nullptr, e, "asg_lsa_batched");
}

int asg_haa_select(const float *beta, const int64_t beta_strides[3], const int64_t *prev,
                   const int64_t prev_strides[2], int64_t B, int n, int m, const double *T_trans_dev, double lambda_,
                   float *col_out, int32_t *status_out, void *hip_stream) {
    if (!beta || !beta_strides || !prev || !prev_strides || !col_out || B < 0 || n <= 0 || m <= 0)
        return fail(nullptr, ASG_E_INVALID_ARG, "asg_haa_select: bad arguments");
    if (n > m) return fail(nullptr, ASG_E_INVALID_ARG, "asg_haa_select: needs n <= m");
    if (m > 1024) return fail(nullptr, ASG_E_INVALID_ARG, "asg_haa_select: m <= 1024");
    if (B == 0) return ASG_OK;
    hipError_t e = asg::launch_haa_select(beta, beta_strides, prev, prev_strides, B, n, m, T_trans_dev, lambda_,
                                          col_out, status_out, static_cast<hipStream_t>(hip_stream));
    return e == hipSuccess ? ASG_OK : hip_fail(nullptr, e, "asg_haa_select");
}

int asg_sap_select(const float *q, const int64_t q_strides[3], int64_t B, int n, int m, double epsilon,
                   uint64_t seed, uint64_t counter, int64_t env_index_base, float *col_out, int32_t *status_out,
                   int32_t *path_steps_out, void *hip_stream) {
    if (!q || !q_strides || !col_out || B < 0 || n <= 0 || m <= 0 || env_index_base < 0)
        return fail(nullptr, ASG_E_INVALID_ARG, "asg_sap_select: bad arguments");
    if (n > m || m > 64) return fail(nullptr, ASG_E_INVALID_ARG, "asg_sap_select: needs n <= m <= 64");
    if (!(epsilon >= 0.0)) return fail(nullptr, ASG_E_INVALID_ARG, "asg_sap_select: epsilon must be >= 0");
    if (B == 0) return ASG_OK;
    hipError_t e = asg::launch_sap_select(q, q_strides, B, n, m, (float)epsilon, seed, (uint32_t)counter,
                                          env_index_base, col_out, status_out, path_steps_out,
                                          static_cast<hipStream_t>(hip_stream));
    return e == hipSuccess ? ASG_OK : hip_fail(nullptr, e, "asg_sap_select");
}

int asg_sap_select_into(const float *q, const int64_t q_strides[3], int64_t B, int n, int m, double epsilon,
                        uint64_t seed, uint64_t counter, int64_t env_index_base, int64_t *act_out,
                        int32_t *status_out, int32_t *path_steps_out, void *hip_stream) {
    if (!q || !q_strides || !act_out || B < 0 || n <= 0 || m <= 0 || env_index_base < 0)
        return fail(nullptr, ASG_E_INVALID_ARG, "asg_sap_select_into: bad arguments");
    if (n > m || m > 64) return fail(nullptr, ASG_E_INVALID_ARG, "asg_sap_select_into: needs n <= m <= 64");
    if (!(epsilon >= 0.0)) return fail(nullptr, ASG_E_INVALID_ARG, "asg_sap_select_into: epsilon must be >= 0");
    if (B == 0) return ASG_OK;
    hipError_t e = asg::launch_sap_select(q, q_strides, B, n, m, (float)epsilon, seed, (uint32_t)counter,
                                          env_index_base, nullptr, status_out, path_steps_out,
                                          static_cast<hipStream_t>(hip_stream), act_out);
    return e == hipSuccess ? ASG_OK : hip_fail(nullptr, e, "asg_sap_select_into");
}

int asg_sap_select_warm(const float *q, const int64_t q_strides[3], int64_t B, int n, int m, double epsilon,
                        uint64_t seed, uint64_t counter, int64_t env_index_base, int64_t *act_out,
                        int32_t *status_out, int32_t *path_steps_out, double *duals, int warm, void *hip_stream) {
    if (!q || !q_strides || !act_out || !duals || B < 0 || n <= 0 || m <= 0 || env_index_base < 0)
        return fail(nullptr, ASG_E_INVALID_ARG, "asg_sap_select_warm: bad arguments");
    if (n > m || m > 64) return fail(nullptr, ASG_E_INVALID_ARG, "asg_sap_select_warm: needs n <= m <= 64");
    if (!(epsilon >= 0.0)) return fail(nullptr, ASG_E_INVALID_ARG, "asg_sap_select_warm: epsilon must be >= 0");
    if ((reinterpret_cast<uintptr_t>(duals) & 7) != 0)
        return fail(nullptr, ASG_E_INVALID_ARG, "asg_sap_select_warm: duals must be 8-B aligned");
    if (B == 0) return ASG_OK;
    hipError_t e = asg::launch_sap_select(q, q_strides, B, n, m, (float)epsilon, seed, (uint32_t)counter,
                                          env_index_base, nullptr, status_out, path_steps_out,
                                          static_cast<hipStream_t>(hip_stream), act_out, duals, warm ? 1 : 0);
    return e == hipSuccess ? ASG_OK : hip_fail(nullptr, e, "asg_sap_select_warm");
}

int asg_sap_noise(const float *q, const int64_t q_strides[3], int64_t B, int n, int m, double epsilon,
                  uint64_t seed, uint64_t counter, int64_t env_index_base, float *q_out, int32_t *status_out,
                  void *hip_stream) {
    if (!q || !q_strides || !q_out || B < 0 || n <= 0 || m <= 0 || env_index_base < 0)
        return fail(nullptr, ASG_E_INVALID_ARG, "asg_sap_noise: bad arguments");
    if (n > m || m > 64) return fail(nullptr, ASG_E_INVALID_ARG, "asg_sap_noise: needs n <= m <= 64");
    if (!(epsilon >= 0.0)) return fail(nullptr, ASG_E_INVALID_ARG, "asg_sap_noise: epsilon must be >= 0");
    if (B == 0) return ASG_OK;
    hipError_t e = asg::launch_sap_noise(q, q_strides, B, n, m, (float)epsilon, seed, (uint32_t)counter,
                                         env_index_base, q_out, status_out, static_cast<hipStream_t>(hip_stream));
    return e == hipSuccess ? ASG_OK : hip_fail(nullptr, e, "asg_sap_noise");
}

int asg_epsilon_greedy(const float *q, const int64_t q_strides[3], const uint8_t *avail,
                       const int64_t avail_strides[3], int64_t B, int n, int m, double epsilon, uint64_t seed,
                       uint64_t counter, int64_t env_index_base, int64_t *out, const int64_t out_strides[2],
                       int32_t *status, void *hip_stream) {
    if (!q || !q_strides || !avail || !avail_strides || !out || !out_strides || B < 0 || n <= 0 || m <= 0 ||
        env_index_base < 0)
        return fail(nullptr, ASG_E_INVALID_ARG, "asg_epsilon_greedy: bad arguments");
    if (!(epsilon >= 0.0 && epsilon <= 1.0))
        return fail(nullptr, ASG_E_INVALID_ARG, "asg_epsilon_greedy: epsilon must be in [0, 1]");
    if (B == 0) return ASG_OK;
    hipError_t e = asg::launch_eps_greedy(q, q_strides, avail, avail_strides, B, n, m, (float)epsilon, seed,
                                          (uint32_t)counter, env_index_base * n, out, out_strides, status,
                                          static_cast<hipStream_t>(hip_stream));
    return e == hipSuccess ? ASG_OK : hip_fail(nullptr, e, "asg_epsilon_greedy");
}

static bool agent_shape_ok(int K, int hidden, int n_out) {
    return hidden == 64 && n_out > 0 && n_out <= 512 && K > 0;
}

int64_t asg_rnn_agent_packed_size(int K, int hidden, int n_out, int use_rnn) {
    if (!agent_shape_ok(K, hidden, n_out)) return fail(nullptr, ASG_E_INVALID_ARG, "bad agent shape");
    return asg::rnn_agent_packed_f4(K, n_out, use_rnn) * 16;
}

int asg_rnn_agent_pack(const float *W1, const float *W_ih, const float *W_hh, const float *W2, int K, int hidden,
                       int n_out, int use_rnn, void *packed, void *hip_stream) {
    if (!W1 || !W_ih || !W2 || !packed || (use_rnn && !W_hh))
        return fail(nullptr, ASG_E_INVALID_ARG, "asg_rnn_agent_pack: NULL weight or output");
    if (!agent_shape_ok(K, hidden, n_out))
        return fail(nullptr, ASG_E_INVALID_ARG,
                    "asg_rnn_agent_pack: needs hidden == 64, 1 <= n_out <= 512, K >= 1");
    hipError_t e = asg::launch_rnn_agent_pack(W1, W_ih, W_hh, W2, K, n_out, use_rnn, static_cast<float4 *>(packed),
                                              static_cast<hipStream_t>(hip_stream));
    return e == hipSuccess ? ASG_OK : hip_fail(nullptr, e, "asg_rnn_agent_pack");
}

int asg_rnn_agent_forward(const float *x, int64_t x_stride, int64_t R, int K, const float *h_in, int64_t h_stride,
                          const void *packed, const float *b1, const float *b_ih, const float *b_hh, const float *b2,
                          int hidden, int n_out, int use_rnn, float *h_out, float *q_out, void *hip_stream) {
    if (!x || !packed || !b1 || !b_ih || !b2 || !h_out || !q_out || R < 0 || (use_rnn && !b_hh))
        return fail(nullptr, ASG_E_INVALID_ARG, "asg_rnn_agent_forward: bad arguments");
    if (!agent_shape_ok(K, hidden, n_out) || (x_stride != 0 && x_stride < K) || h_stride % 4 != 0 ||
        (reinterpret_cast<uintptr_t>(x) % 4) != 0 || (h_in && (reinterpret_cast<uintptr_t>(h_in) % 16) != 0))
        return fail(nullptr, ASG_E_INVALID_ARG,
                    "asg_rnn_agent_forward: needs hidden == 64, 1 <= n_out <= 512, x_stride >= K and 16-B aligned "
                    "h rows");
    if (R == 0) return ASG_OK;
    hipError_t e = asg::launch_rnn_agent_fwd(x, x_stride, R, K, h_in, h_stride, static_cast<const float4 *>(packed),
                                             b1, b_ih, b_hh, b2, n_out, use_rnn, h_out, q_out, nullptr,
                                             static_cast<hipStream_t>(hip_stream));
    return e == hipSuccess ? ASG_OK : hip_fail(nullptr, e, "asg_rnn_agent_forward");
}

int asg_rnn_agent_select(const float *x, int64_t x_stride, int64_t R, int K, const float *h_in, int64_t h_stride,
                         const void *packed, const float *b1, const float *b_ih, const float *b_hh, const float *b2,
                         int hidden, int n_out, int use_rnn, float *h_out, float *q_out, const uint8_t *avail,
                         const int64_t avail_strides[2], int n, double epsilon, uint64_t seed, uint64_t counter,
                         int64_t env_index_base, int64_t *out, const int64_t out_strides[2], int32_t *status,
                         void *hip_stream) {
    if (!x || !packed || !b1 || !b_ih || !b2 || !h_out || !avail || !avail_strides || !out || !out_strides ||
        !status || R < 0 || n <= 0 || env_index_base < 0 || (use_rnn && !b_hh))
        return fail(nullptr, ASG_E_INVALID_ARG, "asg_rnn_agent_select: bad arguments");
    if (!agent_shape_ok(K, hidden, n_out) || (x_stride != 0 && x_stride < K) || h_stride % 4 != 0 ||
        (reinterpret_cast<uintptr_t>(x) % 4) != 0 || (h_in && (reinterpret_cast<uintptr_t>(h_in) % 16) != 0))
        return fail(nullptr, ASG_E_INVALID_ARG, "asg_rnn_agent_select: unsupported shape / alignment");
    if (!(epsilon >= 0.0 && epsilon <= 1.0))
        return fail(nullptr, ASG_E_INVALID_ARG, "asg_rnn_agent_select: epsilon must be in [0, 1]");
    if (R == 0) return ASG_OK;
    hipError_t e = asg::launch_rnn_agent_select(
        x, x_stride, R, K, h_in, h_stride, static_cast<const float4 *>(packed), b1, b_ih, b_hh, b2, n_out, use_rnn,
        h_out, q_out, avail, avail_strides[0], avail_strides[1], n, (float)epsilon, seed, (uint32_t)counter,
        env_index_base * n, out, out_strides[0], out_strides[1], status, static_cast<hipStream_t>(hip_stream));
    return e == hipSuccess ? ASG_OK : hip_fail(nullptr, e, "asg_rnn_agent_select");
}

// ---- filtered selectors (asg_filtered.hip) ------------------------------------------------
int asg_filtered_topm(const void *beta, int beta_dtype, const int64_t beta_strides[4], int64_t B, int n, int m, int L,
                      int M, int64_t *topm_out, void *hip_stream) {
    if (!beta || !beta_strides || !topm_out || B < 0 || n <= 0 || m <= 0 || L <= 0)
        return fail(nullptr, ASG_E_INVALID_ARG, "asg_filtered_topm: bad arguments");
    if (beta_dtype != ASG_F16 && beta_dtype != ASG_F32 && beta_dtype != ASG_F64)
        return fail(nullptr, ASG_E_INVALID_ARG, "asg_filtered_topm: beta must be float16 / float32 / float64");
    if (M <= 0 || M > m) return fail(nullptr, ASG_E_INVALID_ARG, "selected index k out of range");
    if (m > 1024 || M > 64) return fail(nullptr, ASG_E_INVALID_ARG, "asg_filtered_topm: needs m <= 1024, M <= 64");
    if (B == 0) return ASG_OK;
    hipError_t e = asg::launch_filtered_topm(beta, beta_dtype, beta_strides, B, n, m, L, M, topm_out,
                                             static_cast<hipStream_t>(hip_stream));
    return e == hipSuccess ? ASG_OK : hip_fail(nullptr, e, "asg_filtered_topm");
}

static constexpr int kFilteredGaussMaxAgents = (64 * 1024 - 32) / 8;  // 8188

int asg_filtered_benefits(const float *q, const int64_t q_strides[3], const int64_t *topm, int64_t B, int n, int m,
                          int M, const float *tie_noise, double gauss_epsilon, const float *gauss_noise,
                          uint64_t seed, uint64_t counter, int64_t env_index_base, float *mat_out,
                          void *hip_stream) {
    if (!q || !q_strides || !topm || !mat_out || B < 0 || n <= 0 || m <= 0 || env_index_base < 0)
        return fail(nullptr, ASG_E_INVALID_ARG, "asg_filtered_benefits: bad arguments");
    if (M <= 0 || M > m || M > 64 || m > 1024)
        return fail(nullptr, ASG_E_INVALID_ARG, "asg_filtered_benefits: needs 1 <= M <= min(m, 64), m <= 1024");
    if (!(gauss_epsilon >= 0.0)) return fail(nullptr, ASG_E_INVALID_ARG, "asg_filtered_benefits: epsilon >= 0");
    if (B == 0) return ASG_OK;
    hipStream_t s = static_cast<hipStream_t>(hip_stream);
    const bool gauss = gauss_noise != nullptr || gauss_epsilon > 0.0;
    // generated noise: the per-agent |row| sums (8 B each) plus the 32-B partials in LDS, within
    // the 64 KiB a workgroup may hold on every CDNA part (gfx950's 160 KiB not assumed)
    if (gauss && !gauss_noise && n > kFilteredGaussMaxAgents)
        return fail(nullptr, ASG_E_INVALID_ARG, "asg_filtered_benefits: n > 8188 agents with generated Gaussian noise");
    hipError_t e = asg::launch_filtered_matrix(q, q_strides, topm, B, n, m, M, tie_noise, seed, (uint32_t)counter,
                                               env_index_base, mat_out, nullptr, s);
    if (e == hipSuccess && gauss)
        e = asg::launch_filtered_gauss(mat_out, B, n, m, (float)gauss_epsilon, gauss_noise, seed, (uint32_t)counter,
                                       env_index_base, s);
    return e == hipSuccess ? ASG_OK : hip_fail(nullptr, e, "asg_filtered_benefits");
}

int asg_filtered_epsilon_greedy(const float *mat, const int64_t mat_strides[3], const uint8_t *avail,
                                const int64_t avail_strides[3], int64_t B, int n, int m, double epsilon, uint64_t seed,
                                uint64_t counter, int64_t env_index_base, int64_t *out, const int64_t out_strides[2],
                                int32_t *status, void *hip_stream) {
    if (!mat || !mat_strides || !avail || !avail_strides || !out || !out_strides || B < 0 || n <= 0 || m <= 0 ||
        env_index_base < 0)
        return fail(nullptr, ASG_E_INVALID_ARG, "asg_filtered_epsilon_greedy: bad arguments");
    if (!(epsilon >= 0.0 && epsilon <= 1.0))
        return fail(nullptr, ASG_E_INVALID_ARG, "asg_filtered_epsilon_greedy: epsilon must be in [0, 1]");
    if (B == 0) return ASG_OK;
    hipError_t e = asg::launch_eps_greedy(mat, mat_strides, avail, avail_strides, B, n, m, (float)epsilon, seed,
                                          (uint32_t)counter, env_index_base * n, out, out_strides, status,
                                          static_cast<hipStream_t>(hip_stream), /*mask=*/false);
    return e == hipSuccess ? ASG_OK : hip_fail(nullptr, e, "asg_filtered_epsilon_greedy");
}

int asg_filtered_soft_map(const int64_t *picked, const int64_t *topm, int64_t B, int n, int m, int M, uint64_t seed,
                          uint64_t counter, int64_t env_index_base, int64_t *out, int32_t *status, void *hip_stream) {
    if (!picked || !topm || !out || !status || B < 0 || n <= 0 || m <= 0 || env_index_base < 0)
        return fail(nullptr, ASG_E_INVALID_ARG, "asg_filtered_soft_map: bad arguments");
    if (M <= 0 || M >= m) return fail(nullptr, ASG_E_INVALID_ARG, "asg_filtered_soft_map: needs 1 <= M < m");
    if (B == 0) return ASG_OK;
    hipError_t e = asg::launch_filtered_soft_map(picked, topm, B, n, m, M, seed, (uint32_t)counter, env_index_base,
                                                 out, status, static_cast<hipStream_t>(hip_stream));
    return e == hipSuccess ? ASG_OK : hip_fail(nullptr, e, "asg_filtered_soft_map");
}

// ---- fused rollout (asg_h2.hip:rollout_kernel) ------------------------------------------
// field f of a time-major batch ([T+1][E][d2][d3] storage seen as [E][T+1][d2][d3]): the
// row-0 pointer and the row stride (elements), or nullptr when absent / laid out otherwise
static void *tm_base(const asg_field &f, int64_t E, int64_t d2, int64_t d3, int64_t *row, bool *ok) {
    *row = 0;
    if (!f.ptr) return nullptr;
    const bool good = f.stride[0] == d2 * d3 && f.stride[1] == E * d2 * d3 && (d2 == 1 || f.stride[2] == d3) &&
                      (d3 == 1 || f.stride[3] == 1);
    if (!good) *ok = false;
    *row = f.stride[1];
    return f.ptr;
}

int asg_step_select_l2_slices(int n, int m, int L) { return asg::rollout_l2_slices(n, m, L, 1); }
int asg_rollout_l2_slices(int n, int m, int L, int use_rnn) { return asg::rollout_l2_slices(n, m, L, use_rnn); }

// asg_rollout and asg_reset_rollout (reset: the envs' reset runs in the same launch, before
// the selection on row ts)
static int rollout_impl(asg_handle *h, const asg_batch_view *b, int ts, int steps, int select_first, int select_last,
                        int reset, const void *packed, const float *b1, const float *b_r0, const float *b_r1,
                        const float *b2, int K, int hidden, int use_rnn, const float *h_in, int64_t h_stride,
                        float *h_out, double epsilon, uint64_t seed, uint64_t counter, int32_t *status,
                        void *hip_stream, float *q_out = nullptr, int flags = 0) {
    if (!h) return fail(nullptr, ASG_E_INVALID_ARG, "NULL handle");
    if (int rc = check_view(h, b, ts, true)) return rc;
    if (flags & ~ASG_STEP_USE_SELECTED_BIDS) return fail(h, ASG_E_INVALID_ARG, "asg_step_forward_ex: unknown flags");
    if (reset && (flags & ASG_STEP_USE_SELECTED_BIDS))
        return fail(h, ASG_E_INVALID_ARG, "ASG_STEP_USE_SELECTED_BIDS: a reset has no bids row to step");
    if (int rc = selected_bids_ok(h, b, ts, flags)) return rc;
    if (!packed || !b1 || !b_r0 || (use_rnn && !b_r1) || !b2 || !h_out || (!status && !q_out))
        return fail(h, ASG_E_INVALID_ARG, "asg_rollout: NULL agent argument");
    if (q_out && (reinterpret_cast<uintptr_t>(q_out) % 16) != 0)
        return fail(h, ASG_E_INVALID_ARG, "asg_step_forward: q_out must be 16-B aligned");
    const asg::EnvState &st = h->st;
    if (!h->has_reset && !reset) return fail(h, ASG_E_STATE, "step called before reset");
    // the reset inside the launch: Philox bump / dense benefits (the permutation drawn in the
    // kernel), or the MT19937 mode (its draws and table by the reset's draw kernels first, the
    // reset row by the episode launch); not an injected table under Philox
    if (reset && st.rng_mode == ASG_RNG_PHILOX && st.benefit_mode == ASG_BENEFIT_INJECTED)
        return fail(h, ASG_E_INVALID_ARG, "asg_reset_rollout: not with an injected table in the Philox mode (asg_reset)");
    if (reset && st.benefit_mode == ASG_BENEFIT_INJECTED && !h->table_ready)
        return fail(h, ASG_E_STATE, "benefit_mode=injected needs asg_set_benefits before reset");
    const int k0 = reset ? 0 : h->k;
    // steps = 0: asg_reset_forward (the reset and the forward on its row, Q out)
    const bool reset_forward = steps == 0 && reset && q_out;
    if ((steps < 1 && !reset_forward) || k0 + steps > st.T)
        return fail(h, ASG_E_STATE, "asg_rollout: steps must be >= 1 and stay within the episode (k + steps <= T)");
    if (select_first && k0 != 0)
        return fail(h, ASG_E_STATE, "asg_rollout: select_first selects on the reset row (k == 0 only)");
    if (select_last && k0 + steps >= st.T)
        return fail(h, ASG_E_STATE, "asg_rollout: select_last needs a next step to select for (k + steps < T)");
    // the kernel writes batch rows ts .. ts + steps of the [T + 1]-row time-major batch
    if (ts < 0 || ts + steps > st.T)
        return fail(h, ASG_E_INVALID_ARG, "asg_rollout: batch rows ts .. ts + steps must lie in the [T + 1]-row batch");
    // every benefit source: Philox bumps in registers, or the handle's float64 table (MT19937
    // compat / injected), whose reset is asg_reset (above: no asg_reset_rollout)
    if (st.bids && !q_out)
        return fail(h, ASG_E_INVALID_ARG,
                    "asg_rollout: integer actions only (bids_as_actions: asg_step_forward + asg_bids_select)");
    if (hidden != 64 || !asg::rollout_shape_ok(st.n, st.m, st.L, K))
        return fail(h, ASG_E_INVALID_ARG,
                    "asg_rollout: needs the RNNAgent (hidden 64) on the env's obs (K = m (L + 1), L >= 1), "
                    "16 <= m <= 256, n <= 256");
    if (!(epsilon >= 0.0 && epsilon <= 1.0)) return fail(h, ASG_E_INVALID_ARG, "asg_rollout: epsilon in [0, 1]");
    if (h_stride % 4 != 0 || (h_in && (reinterpret_cast<uintptr_t>(h_in) % 16) != 0) ||
        (reinterpret_cast<uintptr_t>(h_out) % 16) != 0)
        return fail(h, ASG_E_INVALID_ARG, "asg_rollout: hidden-state rows must be 16-B aligned");
    const int64_t E = st.E, n = st.n, m = st.m, Kk = K;
    bool ok = true;
    asg::RolloutSlabs sl{};
    sl.obs = static_cast<float *>(tm_base(b->obs, E, n, Kk, &sl.obs_row, &ok));
    sl.beta = static_cast<float *>(tm_base(b->beta, E, n, m, &sl.beta_row, &ok));
    sl.avail = static_cast<uint8_t *>(tm_base(b->avail_actions, E, n, m, &sl.avail_row, &ok));
    sl.onehot = static_cast<int64_t *>(tm_base(b->actions_onehot, E, n, m, &sl.onehot_row, &ok));
    // bids_as_actions: the transition reads the assignments of the bids row (st.assign)
    sl.act = st.bids ? nullptr : static_cast<int64_t *>(tm_base(b->actions, E, n, 1, &sl.act_row, &ok));
    sl.rew = static_cast<float *>(tm_base(b->rewards, E, n, 1, &sl.rew_row, &ok));
    sl.prevb = static_cast<int64_t *>(tm_base(b->prev_assigns, E, n, 1, &sl.prevb_row, &ok));
    sl.term = static_cast<uint8_t *>(tm_base(b->terminated, E, 1, 1, &sl.term_row, &ok));
    sl.filled = static_cast<int64_t *>(tm_base(b->filled, E, 1, 1, &sl.filled_row, &ok));
    auto al = [](const void *p, uintptr_t a) { return (reinterpret_cast<uintptr_t>(p) % a) == 0; };
    if (!ok || !al(sl.obs, 16) || !al(sl.beta, 16) || !al(sl.avail, 16) || !al(sl.onehot, 16))
        return fail(h, ASG_E_INVALID_ARG, "asg_rollout: needs a contiguous time-major batch (EpisodeBatch(time_major=True))");
    DeviceGuard g(h->device);
    hipStream_t s = static_cast<hipStream_t>(hip_stream ? hip_stream : h->stream);
    // as asg_reset: a fresh Philox key per episode, committed once the launch succeeded
    asg::EnvState lst = h->st;
    if (reset && h->has_reset) lst.episode += 1;
    if (st.bids && !reset && !(flags & ASG_STEP_USE_SELECTED_BIDS)) {  // solve the bids of row ts
        hipError_t e0 = asg::launch_bids_assign(*b, st, ts, s);
        if (e0 != hipSuccess) return hip_fail(h, e0, "asg_step_forward (bids LSA)");
    }
    if (reset && st.rng_mode == ASG_RNG_MT19937) {
        hipError_t e0 = asg::launch_reset_draws(lst, !h->constructed, s);
        if (e0 != hipSuccess) return hip_fail(h, e0, "asg_reset_rollout (MT19937 draws)");
    }
    hipError_t e = asg::launch_rollout(sl, lst, ts, k0, steps, select_first, select_last, reset,
                                       static_cast<const float4 *>(packed), b1, b_r0, b_r1, b2, use_rnn, h_in, h_stride,
                                       h_out, q_out, (float)epsilon, seed, (uint32_t)counter, st.env_base * n, status, s);
    if (e != hipSuccess) return hip_fail(h, e, "asg_rollout");
    h->st.episode = lst.episode;
    if (reset) {
        h->constructed = true;
        h->has_reset = true;
    }
    h->k = k0 + steps;
    h->bids_tag = {};
    return ASG_OK;
}

int asg_rollout(asg_handle *h, const asg_batch_view *b, int ts, int steps, int select_first, int select_last,
                const void *packed, const float *b1, const float *b_r0, const float *b_r1, const float *b2, int K,
                int hidden, int use_rnn, const float *h_in, int64_t h_stride, float *h_out, double epsilon,
                uint64_t seed, uint64_t counter, int32_t *status, void *hip_stream) {
    return rollout_impl(h, b, ts, steps, select_first, select_last, 0, packed, b1, b_r0, b_r1, b2, K, hidden, use_rnn,
                        h_in, h_stride, h_out, epsilon, seed, counter, status, hip_stream);
}

int asg_reset_rollout(asg_handle *h, const asg_batch_view *b, int ts, int steps, int select_last, const void *packed,
                      const float *b1, const float *b_r0, const float *b_r1, const float *b2, int K, int hidden,
                      int use_rnn, const float *h_in, int64_t h_stride, float *h_out, double epsilon, uint64_t seed,
                      uint64_t counter, int32_t *status, void *hip_stream) {
    return rollout_impl(h, b, ts, steps, 1, select_last, 1, packed, b1, b_r0, b_r1, b2, K, hidden, use_rnn, h_in,
                        h_stride, h_out, epsilon, seed, counter, status, hip_stream);
}

int asg_step_select(asg_handle *h, const asg_batch_view *b, int ts, const void *packed, const float *b1,
                    const float *b_ih, const float *b_hh, const float *b2, int K, int hidden, const float *h_in,
                    int64_t h_stride, float *h_out, double epsilon, uint64_t seed, uint64_t counter,
                    int32_t *status, void *hip_stream) {
    return asg_rollout(h, b, ts, 1, 0, 1, packed, b1, b_ih, b_hh, b2, K, hidden, 1, h_in, h_stride, h_out, epsilon,
                       seed, counter, status, hip_stream);
}

int asg_reset_forward(asg_handle *h, const asg_batch_view *b, int ts, const void *packed, const float *b1,
                      const float *b_r0, const float *b_r1, const float *b2, int K, int hidden, int use_rnn,
                      const float *h_in, int64_t h_stride, float *h_out, float *q_out, void *hip_stream) {
    if (!q_out) return fail(h, ASG_E_INVALID_ARG, "asg_reset_forward: NULL q_out");
    return rollout_impl(h, b, ts, 0, 1, 1, 1, packed, b1, b_r0, b_r1, b2, K, hidden, use_rnn, h_in, h_stride, h_out,
                        0.0, 0, 0, nullptr, hip_stream, q_out);
}

int asg_step_forward(asg_handle *h, const asg_batch_view *b, int ts, const void *packed, const float *b1,
                     const float *b_r0, const float *b_r1, const float *b2, int K, int hidden, int use_rnn,
                     const float *h_in, int64_t h_stride, float *h_out, float *q_out, void *hip_stream) {
    return asg_step_forward_ex(h, b, ts, packed, b1, b_r0, b_r1, b2, K, hidden, use_rnn, h_in, h_stride, h_out, q_out,
                               0, hip_stream);
}

int asg_step_forward_ex(asg_handle *h, const asg_batch_view *b, int ts, const void *packed, const float *b1,
                        const float *b_r0, const float *b_r1, const float *b2, int K, int hidden, int use_rnn,
                        const float *h_in, int64_t h_stride, float *h_out, float *q_out, int flags,
                        void *hip_stream) {
    if (!q_out) return fail(h, ASG_E_INVALID_ARG, "asg_step_forward: NULL q_out");
    return rollout_impl(h, b, ts, 1, 0, 1, 0, packed, b1, b_r0, b_r1, b2, K, hidden, use_rnn, h_in, h_stride, h_out,
                        0.0, 0, 0, nullptr, hip_stream, q_out, flags);
}

int asg_bids_select(asg_handle *h, const float *q, const int64_t q_strides[3], float *bids_out,
                    const int64_t out_strides[3], int row_softmax, int col_softmax, double stdv, uint64_t seed,
                    uint64_t counter, void *hip_stream) {
    return asg_bids_select_count(h, q, q_strides, bids_out, out_strides, row_softmax, col_softmax, stdv, seed, counter,
                                 nullptr, hip_stream);
}

int asg_bids_select_count(asg_handle *h, const float *q, const int64_t q_strides[3], float *bids_out,
                          const int64_t out_strides[3], int row_softmax, int col_softmax, double stdv, uint64_t seed,
                          uint64_t counter, int32_t *path_steps_out, void *hip_stream) {
    if (!h) return fail(nullptr, ASG_E_INVALID_ARG, "NULL handle");
    const EnvState &st = h->st;
    if (!st.bids) return fail(h, ASG_E_INVALID_ARG, "asg_bids_select: the handle was not created with bids_as_actions");
    if (!q || !q_strides || !bids_out || !out_strides) return fail(h, ASG_E_INVALID_ARG, "asg_bids_select: NULL argument");
    if (st.m > 64) return fail(h, ASG_E_INVALID_ARG, "asg_bids_select: m <= 64 (register-resident bids)");
    if (!(stdv >= 0.0 && stdv < 1e30)) return fail(h, ASG_E_INVALID_ARG, "asg_bids_select: std must be finite and >= 0");
    DeviceGuard g(h->device);
    hipStream_t s = static_cast<hipStream_t>(hip_stream ? hip_stream : h->stream);
    hipError_t e = asg::launch_bids_select(q, q_strides, st.E, st.n, st.m, row_softmax != 0, col_softmax != 0,
                                           (float)stdv, seed, (uint32_t)counter, st.env_base, bids_out, out_strides,
                                           st.assign, st.err, s, path_steps_out);
    if (e != hipSuccess) return hip_fail(h, e, "asg_bids_select");
    h->bids_tag.row = bids_out;
    h->bids_tag.s_env = out_strides[0];
    h->bids_tag.s_agent = out_strides[1];
    h->bids_tag.s_task = out_strides[2];
    return ASG_OK;
}

}  // extern "C"


