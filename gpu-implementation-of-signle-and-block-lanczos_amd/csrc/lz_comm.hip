// lz_comm.hip -- RCCL and in-process (virtual-rank) implementations of the
// exchange layer (lz_comm.hpp), and their C-ABI entry points.
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "lz_comm.hpp"

namespace lz {

#define LZ_NCCL_CHECK(expr)                                                          \
    do {                                                                             \
        ncclResult_t r_ = (expr);                                                    \
        if (r_ != ncclSuccess) {                                                     \
            ::lz::set_error("%s -> %s", #expr, ncclGetErrorString(r_));             \
            return LZ_E_COMM;                                                        \
        }                                                                            \
    } while (0)

// ------------------------------------------------------------------ RCCL
class RcclComm final : public Comm {
public:
    ncclComm_t c = nullptr;
    ~RcclComm() override
    {
        if (c) ncclCommDestroy(c);
    }
    bool aborted = false;
    const char *kind() const override { return "rccl"; }
    // a failing rank aborts its communicator: this rank's RCCL operations in
    // flight on it return, and every later call here fails (lz_comm_destroy and
    // a new lz_comm_init with a new unique id make the handle usable again).
    // Peers blocked in a collective with this rank are released only if they
    // poll ncclCommGetAsyncError or abort their own communicator.
    void abort() override
    {
        if (c && !aborted) (void)ncclCommAbort(c);
        if (c) c = nullptr;
        aborted = true;
    }
    int usable() const
    {
        if (!c || aborted) {
            set_error("RCCL communicator aborted");
            return LZ_E_COMM;
        }
        return LZ_OK;
    }
    int allreduce_sum(double *buf, size_t count, hipStream_t s) override
    {
        LZ_TRY(usable());
        ++issued;
        LZ_NCCL_CHECK(ncclAllReduce(buf, buf, count, ncclDouble, ncclSum, c, s));
        return LZ_OK;
    }
    int allgather(const void *send, void *X, size_t slot_bytes, hipStream_t s) override
    {
        // in place when send is this rank's slot (RCCL then copies nothing locally)
        LZ_TRY(usable());
        ++issued;
        if (slot_bytes % 8 == 0)
            LZ_NCCL_CHECK(ncclAllGather(send, X, slot_bytes / 8, ncclDouble, c, s));
        else
            LZ_NCCL_CHECK(ncclAllGather(send, X, slot_bytes, ncclChar, c, s));
        return LZ_OK;
    }
    int exchange(const P2POp *ops, int nops, hipStream_t s) override
    {
        LZ_TRY(usable());
        ++issued;
        LZ_NCCL_CHECK(ncclGroupStart());
        ncclResult_t r = ncclSuccess;
        for (int i = 0; i < nops && r == ncclSuccess; ++i) {
            const P2POp &o = ops[i];
            if (o.peer == rank) continue;
            if (o.send_bytes) r = ncclSend(o.send, o.send_bytes, ncclChar, o.peer, c, s);
            if (o.recv_bytes && r == ncclSuccess) r = ncclRecv(o.recv, o.recv_bytes, ncclChar, o.peer, c, s);
        }
        const ncclResult_t e = ncclGroupEnd();
        LZ_NCCL_CHECK(r);
        LZ_NCCL_CHECK(e);
        return LZ_OK;
    }
};

int make_rccl_comm(int nranks, int rank, const unsigned char id[128], Comm **out)
{
    static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId size");
    ncclUniqueId uid;
    std::memcpy(&uid, id, 128);
    RcclComm *rc = new RcclComm();
    rc->nranks = nranks;
    rc->rank = rank;
    const ncclResult_t r = ncclCommInitRank(&rc->c, nranks, uid, rank);
    if (r != ncclSuccess) {
        rc->c = nullptr;
        delete rc;
        set_error("ncclCommInitRank -> %s", ncclGetErrorString(r));
        return LZ_E_COMM;
    }
    *out = rc;
    return LZ_OK;
}

// ------------------------------------------------------ virtual ranks
// The group's shared state.  Host data published for collective k lives in
// pub[k & 1], so a slow peer still reading collective k's entries never sees
// collective k+1's (it reads them before arriving at barrier k+1).
struct LocalGroupState {
    int n = 0, device = 0;
    std::mutex mu;
    std::condition_variable cv;
    int arrived = 0;
    uint64_t gen = 0;
    bool aborted = false;
    std::string why;
    double timeout_s = 300.0;
    static constexpr size_t kStage = 4096;  // doubles per rank and parity (b x b slabs, b <= 64)
    double *staging = nullptr;              // device: [2][n][kStage]
    enum Op { OP_NONE = -1, OP_ALLREDUCE = 0, OP_ALLGATHER = 1, OP_EXCHANGE = 2, OP_FENCE = 3 };
    struct Pub {
        int op = OP_NONE;
        uint64_t seq = 0;
        const void *send = nullptr;
        size_t bytes = 0;
        std::vector<P2POp> ops;
    };
    struct Slot {
        bool attached = false;
        hipEvent_t ready[2] = {nullptr, nullptr}, done[2] = {nullptr, nullptr};
        Pub pub[2];
    };
    std::vector<Slot> slot;

    ~LocalGroupState()
    {
        if (staging) {
            (void)hipSetDevice(device);
            (void)hipFree(staging);
        }
    }

    void abort(const char *reason)
    {
        std::lock_guard<std::mutex> lk(mu);
        if (!aborted) why = reason;
        aborted = true;
        cv.notify_all();
    }

    // every attached rank arrives; a timeout or an abort ends it for all
    int barrier(int rank, const char *what)
    {
        std::unique_lock<std::mutex> lk(mu);
        if (aborted) {
            set_error("local group: %s on rank %d after abort (%s)", what, rank, why.c_str());
            return LZ_E_COMM;
        }
        const uint64_t my = gen;
        if (++arrived == n) {
            arrived = 0;
            ++gen;
            cv.notify_all();
            return LZ_OK;
        }
        const auto limit = std::chrono::duration<double>(timeout_s);
        const bool ok = cv.wait_for(lk, limit, [&] { return gen != my || aborted; });
        if (gen != my) return LZ_OK;
        if (!ok && !aborted) {
            aborted = true;
            why = std::string("timeout in ") + what;
            cv.notify_all();
        }
        set_error("local group: %s on rank %d: %s", what, rank, why.c_str());
        return LZ_E_COMM;
    }
};

// out[i] = sum over ranks r = 0..n-1, in rank order, of stage[r * stride + i]
__global__ void k_sum_ranks(size_t count, const double *__restrict__ stage, int n, size_t stride,
                            double *__restrict__ out)
{
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < count; i += (size_t)gridDim.x * blockDim.x) {
        double s = stage[i];
        for (int r = 1; r < n; ++r) s += stage[r * stride + i];
        out[i] = s;
    }
}

class LocalComm final : public Comm {
public:
    std::shared_ptr<LocalGroupState> g;
    uint64_t seq = 0;
    int par = 0;  // parity of the collective in progress

    ~LocalComm() override
    {
        if (!g) return;
        auto &sl = g->slot[rank];
        {
            std::lock_guard<std::mutex> lk(g->mu);
            sl.attached = false;
        }
        for (int k = 0; k < 2; ++k) {
            if (sl.ready[k]) (void)hipEventDestroy(sl.ready[k]);
            if (sl.done[k]) (void)hipEventDestroy(sl.done[k]);
            sl.ready[k] = sl.done[k] = nullptr;
        }
    }
    const char *kind() const override { return "local"; }
    void abort() override { g->abort("aborted by a rank"); }
    bool abort_wakes_peers() const override { return true; }

    int begin(int op, const void *send, size_t bytes, const P2POp *ops, int nops, hipStream_t s)
    {
        ++issued;
        par = (int)(seq & 1);
        auto &me = g->slot[rank];
        LocalGroupState::Pub &p = me.pub[par];
        p.op = op;
        p.seq = seq;
        p.send = send;
        p.bytes = bytes;
        p.ops.assign(ops, ops + nops);
        LZ_HIP_TRY(hipEventRecord(me.ready[par], s));
        LZ_TRY(g->barrier(rank, "collective"));
        for (int q = 0; q < nranks; ++q) {
            if (q == rank) continue;
            const auto &pq = g->slot[q].pub[par];
            if (pq.op != op || pq.seq != seq) {
                g->abort("collective mismatch");
                set_error("local group: rank %d issued collective %d (#%llu), rank %d issued %d (#%llu)", rank, op,
                          (unsigned long long)seq, q, pq.op, (unsigned long long)pq.seq);
                return LZ_E_COMM;
            }
            LZ_HIP_TRY(hipStreamWaitEvent(s, g->slot[q].ready[par], 0));
            LZ_HIP_TRY(hipStreamWaitEvent(s, g->slot[q].done[par ^ 1], 0));
        }
        return LZ_OK;
    }
    int end(hipStream_t s)
    {
        LZ_HIP_TRY(hipEventRecord(g->slot[rank].done[par], s));
        ++seq;
        return LZ_OK;
    }

    int allreduce_sum(double *buf, size_t count, hipStream_t s) override
    {
        LZ_ARG_CHECK(count <= LocalGroupState::kStage, "local all-reduce: count <= 4096 doubles");
        const size_t stride = LocalGroupState::kStage;
        double *base = g->staging + (size_t)(seq & 1) * g->n * stride;
        LZ_HIP_TRY(hipMemcpyAsync(base + rank * stride, buf, count * sizeof(double), hipMemcpyDeviceToDevice, s));
        LZ_TRY(begin(LocalGroupState::OP_ALLREDUCE, nullptr, count, nullptr, 0, s));
        const int grid = (int)std::max<size_t>(1, std::min<size_t>((count + 255) / 256, 64));
        hipLaunchKernelGGL(k_sum_ranks, dim3(grid), dim3(256), 0, s, count, (const double *)base, nranks, stride, buf);
        LZ_LAUNCH_CHECK();
        return end(s);
    }
    int allgather(const void *send, void *X, size_t slot_bytes, hipStream_t s) override
    {
        LZ_TRY(begin(LocalGroupState::OP_ALLGATHER, send, slot_bytes, nullptr, 0, s));
        char *xb = static_cast<char *>(X);
        for (int q = 0; q < nranks; ++q) {
            const auto &pq = g->slot[q].pub[par];
            if (q != rank && pq.bytes != slot_bytes) {
                g->abort("all-gather size mismatch");
                set_error("local all-gather: rank %d slot %zu bytes, rank %d %zu", rank, slot_bytes, q, pq.bytes);
                return LZ_E_COMM;
            }
            const void *src = q == rank ? send : pq.send;
            char *dst = xb + (size_t)q * slot_bytes;
            if (src != dst && slot_bytes)
                LZ_HIP_TRY(hipMemcpyAsync(dst, src, slot_bytes, hipMemcpyDeviceToDevice, s));
        }
        return end(s);
    }
    int exchange(const P2POp *ops, int nops, hipStream_t s) override
    {
        LZ_TRY(begin(LocalGroupState::OP_EXCHANGE, nullptr, 0, ops, nops, s));
        for (int i = 0; i < nops; ++i) {
            const P2POp &o = ops[i];
            if (o.peer == rank || o.recv_bytes == 0) continue;
            const auto &pq = g->slot[o.peer].pub[par];
            const P2POp *match = nullptr;
            for (const P2POp &x : pq.ops)
                if (x.peer == rank) match = &x;
            if (!match || match->send_bytes != o.recv_bytes) {
                g->abort("exchange mismatch");
                set_error("local exchange: rank %d expects %zu bytes from rank %d, which sends %zu", rank, o.recv_bytes,
                          o.peer, match ? match->send_bytes : (size_t)0);
                return LZ_E_COMM;
            }
            LZ_HIP_TRY(hipMemcpyAsync(o.recv, match->send, o.recv_bytes, hipMemcpyDeviceToDevice, s));
        }
        return end(s);
    }
    int fence(hipStream_t s) override
    {
        LZ_TRY(begin(LocalGroupState::OP_FENCE, nullptr, 0, nullptr, 0, s));
        return end(s);
    }
};

}  // namespace lz

struct lz_local_group {
    std::shared_ptr<lz::LocalGroupState> st;
};

using namespace lz;

extern "C" {

int lz_local_group_create(int device, int nranks, lz_local_group **out)
{
    LZ_ARG_CHECK(out != nullptr && nranks >= 1 && nranks <= 64, "local group: 1 <= nranks <= 64");
    *out = nullptr;
    LZ_HIP_TRY(hipSetDevice(device));
    auto st = std::make_shared<LocalGroupState>();
    st->n = nranks;
    st->device = device;
    st->slot.resize(nranks);
    if (const char *t = getenv("LZ_LOCAL_TIMEOUT_S"); t && atof(t) > 0) st->timeout_s = atof(t);
    LZ_HIP_TRY(hipMalloc(&st->staging, sizeof(double) * 2 * nranks * LocalGroupState::kStage));
    *out = new lz_local_group{st};
    return LZ_OK;
}

int lz_local_group_destroy(lz_local_group *g)
{
    delete g;  // the state lives on while a handle still holds it
    return LZ_OK;
}

int lz_local_group_abort(lz_local_group *g)
{
    LZ_ARG_CHECK(g != nullptr, "group is NULL");
    g->st->abort("lz_local_group_abort");
    return LZ_OK;
}

int lz_comm_init_local(lz_handle *h, lz_local_group *grp, int rank)
{
    LZ_ARG_CHECK(h && grp, "NULL handle / group");
    auto &st = grp->st;
    LZ_ARG_CHECK(rank >= 0 && rank < st->n, "rank in [0, nranks)");
    LZ_ARG_CHECK(h->device == st->device, "the group's ranks share one device");
    LZ_ARG_CHECK(h->comm == nullptr, "handle already has a communicator (lz_comm_destroy first)");
    LZ_HIP_TRY(hipSetDevice(h->device));
    {
        std::lock_guard<std::mutex> lk(st->mu);
        LZ_ARG_CHECK(!st->slot[rank].attached, "rank already attached");
        st->slot[rank].attached = true;
    }
    LocalComm *c = new LocalComm();  // its destructor detaches the rank and frees the events
    c->g = st;
    c->nranks = st->n;
    c->rank = rank;
    auto make_events = [&]() -> int {
        auto &sl = st->slot[rank];
        for (int k = 0; k < 2; ++k) {
            LZ_HIP_TRY(hipEventCreateWithFlags(&sl.ready[k], hipEventDisableTiming));
            LZ_HIP_TRY(hipEventCreateWithFlags(&sl.done[k], hipEventDisableTiming));
            // recorded once, so the first collectives' waits on them are satisfied
            LZ_HIP_TRY(hipEventRecord(sl.ready[k], h->stream));
            LZ_HIP_TRY(hipEventRecord(sl.done[k], h->stream));
        }
        LZ_HIP_TRY(hipStreamSynchronize(h->stream));
        return LZ_OK;
    };
    int rc = make_events();
    if (rc == LZ_OK) rc = attach_comm(h, c);  // owns c from here, also on failure
    else delete c;
    // the ranks share the device: a kernel whose blocks wait on each other (the
    // wavefront step) gets a share of the CUs so every rank's grid is resident
    if (rc == LZ_OK) h->grid_cap = std::max(1, h->n_cu / st->n);
    return rc;
}

int lz_comm_unique_id(unsigned char out[128])
{
    ncclUniqueId id;
    LZ_NCCL_CHECK(ncclGetUniqueId(&id));
    std::memcpy(out, &id, 128);
    return LZ_OK;
}

int lz_comm_abort(lz_handle *h)
{
    LZ_ARG_CHECK(h != nullptr, "handle is NULL");
    if (h->comm) h->comm->abort();
    return LZ_OK;
}

}  // extern "C"
