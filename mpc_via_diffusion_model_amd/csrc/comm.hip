// Communicators of the candidate-batch exchange (comm.h): RCCL over xGMI, and an in-process loopback
// group of virtual ranks on one device. Host code plus one small reduction kernel.
#include <hip/hip_runtime.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <map>
#include <mutex>
#include <vector>

#include <rccl/rccl.h>

#include "../../include/mpcd.h"
#include "comm.h"

namespace {

#define C_HIP(expr)                                                                    \
    do {                                                                               \
        hipError_t e_ = (expr);                                                        \
        if (e_ != hipSuccess) {                                                        \
            err = std::string(#expr ": ") + hipGetErrorString(e_);                     \
            return MPCD_EHIP;                                                          \
        }                                                                              \
    } while (0)
#define C_NCCL(expr)                                                                   \
    do {                                                                               \
        ncclResult_t r_ = (expr);                                                      \
        if (r_ != ncclSuccess) {                                                       \
            err = std::string(#expr ": ") + ncclGetErrorString(r_);                    \
            return MPCD_EHIP;                                                          \
        }                                                                              \
    } while (0)

struct RcclComm final : Comm {
    ncclComm_t c = nullptr;
    ~RcclComm() override
    {
        if (c) (void)ncclCommDestroy(c);
    }
    int allgather(const void *send, void *recv, size_t bytes, hipStream_t st, std::string &err) override
    {
        C_NCCL(ncclAllGather(send, recv, bytes, ncclInt8, c, st));  // type-agnostic: gather bytes
        return MPCD_OK;
    }
    int allreduce(void *buf, size_t count, CommOp op, hipStream_t st, std::string &err) override
    {
        if (op == COMM_SUM_F32) C_NCCL(ncclAllReduce(buf, buf, count, ncclFloat32, ncclSum, c, st));
        else C_NCCL(ncclAllReduce(buf, buf, count, ncclInt32, ncclMax, c, st));
        return MPCD_OK;
    }
    int broadcast(void *buf, size_t bytes, int root, hipStream_t st, std::string &err) override
    {
        C_NCCL(ncclBroadcast(buf, buf, bytes, ncclInt8, root, c, st));
        return MPCD_OK;
    }
};

// ---- loopback group: rendezvous of the member threads + per-rank HIP events
struct LoopGroup {
    int n = 0, members = 0;
    std::mutex mu;
    std::condition_variable cv;
    int arrived = 0;
    uint64_t gen = 0;
    bool broken = false;  // a member timed out: the phases can no longer pair up, every later call fails
    std::vector<const void *> src;
    std::vector<hipEvent_t> ready, copied;  // owned by the member ranks
    std::vector<bool> joined;

    // every member thread must call; false on timeout (a peer that never arrives) and on every call after
    // one: a timed-out member has left the generation its arrival counted in, so a late peer would release
    // it and the next collective would pair mismatched phases (stale buffers) instead of failing
    bool barrier()
    {
        std::unique_lock<std::mutex> lk(mu);
        if (broken) return false;
        const uint64_t g = gen;
        if (++arrived == n) {
            arrived = 0;
            ++gen;
            cv.notify_all();
            return true;
        }
        if (cv.wait_for(lk, std::chrono::seconds(120), [&] { return gen != g || broken; }) && !broken) return true;
        broken = true;
        cv.notify_all();
        return false;
    }
};

std::mutex g_reg_mu;
std::map<uint64_t, LoopGroup *> g_groups;

__global__ void reduce_ranks_kernel(const void *scratch, void *out, size_t count, int n, int op)
{
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < count; i += (size_t)gridDim.x * blockDim.x) {
        if (op == COMM_SUM_F32) {
            const float *s = static_cast<const float *>(scratch);
            float v = s[i];
            for (int p = 1; p < n; ++p) v = v + s[(size_t)p * count + i];
            static_cast<float *>(out)[i] = v;
        } else {
            const int *s = static_cast<const int *>(scratch);
            int v = s[i];
            for (int p = 1; p < n; ++p) v = max(v, s[(size_t)p * count + i]);
            static_cast<int *>(out)[i] = v;
        }
    }
}

struct LoopbackComm final : Comm {
    uint64_t key = 0;
    LoopGroup *g = nullptr;
    void *scratch = nullptr;
    size_t scratch_bytes = 0;

    ~LoopbackComm() override
    {
        if (scratch) (void)hipFree(scratch);
        if (!g) return;
        std::lock_guard<std::mutex> lk(g_reg_mu);
        (void)hipEventDestroy(g->ready[rank]);
        (void)hipEventDestroy(g->copied[rank]);
        g->joined[rank] = false;
        if (--g->members == 0) {
            g_groups.erase(key);
            delete g;
        }
    }

    int rendezvous(std::string &err)
    {
        if (!g->barrier()) {
            err = "loopback communicator: a peer rank did not reach a collective within 120 s (the group is "
                  "unusable from then on)";
            return MPCD_ESTATE;
        }
        return MPCD_OK;
    }

    // phase 1: publish `src` once this stream has produced it, wait for every peer's publication
    int publish(const void *src, hipStream_t st, std::string &err)
    {
        C_HIP(hipEventRecord(g->ready[rank], st));
        g->src[rank] = src;
        return rendezvous(err);
    }
    // phase 2: this rank's reads of the peers are enqueued; nobody continues (e.g. overwrites its
    // published buffer) on its stream until every peer's reads have run
    int retire(hipStream_t st, std::string &err)
    {
        C_HIP(hipEventRecord(g->copied[rank], st));
        int rc = rendezvous(err);
        if (rc) return rc;
        for (int p = 0; p < nranks; ++p)
            if (p != rank) C_HIP(hipStreamWaitEvent(st, g->copied[p], 0));
        return MPCD_OK;
    }

    int allgather(const void *send, void *recv, size_t bytes, hipStream_t st, std::string &err) override
    {
        int rc = publish(send, st, err);
        if (rc) return rc;
        for (int p = 0; p < nranks; ++p) {
            if (p != rank) C_HIP(hipStreamWaitEvent(st, g->ready[p], 0));
            C_HIP(hipMemcpyAsync(static_cast<char *>(recv) + (size_t)p * bytes, g->src[p], bytes, hipMemcpyDeviceToDevice, st));
        }
        return retire(st, err);
    }

    int allreduce(void *buf, size_t count, CommOp op, hipStream_t st, std::string &err) override
    {
        const size_t bytes = count * 4;
        if (scratch_bytes < bytes * nranks) {
            if (scratch) (void)hipFree(scratch);
            scratch = nullptr;
            scratch_bytes = 0;
            C_HIP(hipMalloc(&scratch, bytes * nranks));
            scratch_bytes = bytes * nranks;
        }
        int rc = publish(buf, st, err);
        if (rc) return rc;
        for (int p = 0; p < nranks; ++p) {
            if (p != rank) C_HIP(hipStreamWaitEvent(st, g->ready[p], 0));
            C_HIP(hipMemcpyAsync(static_cast<char *>(scratch) + (size_t)p * bytes, g->src[p], bytes, hipMemcpyDeviceToDevice, st));
        }
        if ((rc = retire(st, err))) return rc;  // every peer has copied our buf: now overwrite it
        const unsigned blocks = (unsigned)std::min<size_t>(1024, (count + 255) / 256);
        hipLaunchKernelGGL(reduce_ranks_kernel, dim3(blocks ? blocks : 1), dim3(256), 0, st, scratch, buf, count, nranks,
                           (int)op);
        C_HIP(hipGetLastError());
        return MPCD_OK;
    }

    int broadcast(void *buf, size_t bytes, int root, hipStream_t st, std::string &err) override
    {
        int rc = publish(buf, st, err);
        if (rc) return rc;
        if (rank != root) {
            C_HIP(hipStreamWaitEvent(st, g->ready[root], 0));
            C_HIP(hipMemcpyAsync(buf, g->src[root], bytes, hipMemcpyDeviceToDevice, st));
        }
        return retire(st, err);
    }
};

}  // namespace

int comm_unique_id(void *id_out, std::string &err)
{
    static_assert(sizeof(ncclUniqueId) == MPCD_COMM_ID_BYTES, "ncclUniqueId size");
    ncclUniqueId id;
    C_NCCL(ncclGetUniqueId(&id));
    memcpy(id_out, &id, sizeof id);
    return MPCD_OK;
}

int comm_create_rccl(int nranks, int rank, const void *id_in, Comm **out, std::string &err)
{
    ncclUniqueId id;
    memcpy(&id, id_in, sizeof id);
    auto *c = new RcclComm();
    ncclResult_t r = ncclCommInitRank(&c->c, nranks, id, rank);
    if (r != ncclSuccess) {
        c->c = nullptr;
        delete c;
        err = std::string("ncclCommInitRank: ") + ncclGetErrorString(r);
        return MPCD_EHIP;
    }
    c->nranks = nranks;
    c->rank = rank;
    *out = c;
    return MPCD_OK;
}

int comm_create_loopback(int nranks, int rank, uint64_t key, Comm **out, std::string &err)
{
    std::lock_guard<std::mutex> lk(g_reg_mu);
    LoopGroup *g;
    auto it = g_groups.find(key);
    if (it == g_groups.end()) {
        g = new LoopGroup();
        g->n = nranks;
        g->src.assign(nranks, nullptr);
        g->ready.assign(nranks, nullptr);
        g->copied.assign(nranks, nullptr);
        g->joined.assign(nranks, false);
        g_groups[key] = g;
    } else {
        g = it->second;
    }
    if (g->n != nranks) {
        err = "loopback group " + std::to_string(key) + " has " + std::to_string(g->n) + " ranks, not " + std::to_string(nranks);
        return MPCD_EINVAL;
    }
    if (g->joined[rank]) {
        err = "loopback group " + std::to_string(key) + ": rank " + std::to_string(rank) + " joined twice";
        return MPCD_ESTATE;
    }
    hipEvent_t a = nullptr, b = nullptr;
    if (hipEventCreateWithFlags(&a, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&b, hipEventDisableTiming) != hipSuccess) {
        if (a) (void)hipEventDestroy(a);
        if (g->members == 0) {
            g_groups.erase(key);
            delete g;
        }
        err = "hipEventCreate failed";
        return MPCD_EHIP;
    }
    g->ready[rank] = a;
    g->copied[rank] = b;
    g->joined[rank] = true;
    ++g->members;
    auto *c = new LoopbackComm();
    c->nranks = nranks;
    c->rank = rank;
    c->key = key;
    c->g = g;
    *out = c;
    return MPCD_OK;
}
