// lz_comm.hpp -- the exchange layer of the row-partitioned iteration.
//
// The distributed block Lanczos (lz_api.hip) needs three collective shapes per
// step: a sum of b x b fp64 partial Grams (all-reduce), the Krylov block's
// all-gather (the north star's exchange) or a grouped point-to-point round
// (halo rows).  They go through this interface, with two implementations:
//
//   RcclComm   one process per GPU, RCCL over xGMI (ncclAllReduce,
//              ncclAllGather, grouped ncclSend/ncclRecv).  The production path.
//   LocalComm  N "virtual ranks" in ONE process on one device, one host thread
//              and one stream per rank (lz_local_group_create /
//              lz_comm_init_local).  Each collective publishes the rank's
//              buffers, meets the others at a host barrier, then PULLS the
//              peers' data with device copies on its own stream behind the
//              peers' ready events.  It exists so one GPU can run an N-rank
//              decomposition through the very same native iteration (packing,
//              compact-column pass 1, SWAP pass 2, all-reduce slots) that
//              RCCL ranks run; the tests compare it with the oracle at N = 2,
//              4, 8.
//
// Ordering contract of LocalComm (every collective k of a rank, on stream s):
//   publish -> record ready[k&1] -> host barrier -> wait every peer's
//   ready[k&1] and done[(k-1)&1] -> pull -> record done[k&1].
// A rank writes a buffer its peers read in collective k only after collective
// k+1's barrier (the algorithm's own order: a slot read by an all-gather is
// rewritten by pass 2 after the next all-reduce), so waiting on the peers'
// previous done events orders those writes behind the reads.
#pragma once
#include <cstddef>
#include <cstdint>

#include "lz_common.hpp"

namespace lz {

struct P2POp {
    int peer;
    const void *send;   // bytes this rank sends to `peer` (may be null when send_bytes == 0)
    size_t send_bytes;
    void *recv;         // where the bytes from `peer` land
    size_t recv_bytes;
};

class Comm {
public:
    int nranks = 1, rank = 0;
    uint64_t issued = 0;  // collectives issued so far (a failure after one aborts, dist_solve)
    virtual ~Comm() = default;
    virtual const char *kind() const = 0;
    // in place sum of count doubles over the ranks; every rank gets the same bits
    virtual int allreduce_sum(double *buf, size_t count, hipStream_t s) = 0;
    // slot g (slot_bytes at X + g * slot_bytes) <- rank g's `send`; send may be
    // this rank's own slot of X (in place)
    virtual int allgather(const void *send, void *X, size_t slot_bytes, hipStream_t s) = 0;
    // one grouped point-to-point round (every op: send to / receive from op.peer)
    virtual int exchange(const P2POp *ops, int nops, hipStream_t s) = 0;
    // after the fence completes on s no peer reads this rank's buffers any more
    virtual int fence(hipStream_t s)
    {
        (void)s;
        return LZ_OK;
    }
    // wake every rank blocked in a collective of this group with an error; for
    // RCCL this is ncclCommAbort, after which the communicator is unusable
    virtual void abort() {}
    // whether abort() releases peers that wait for a collective this rank never
    // issued (a virtual-rank group's host barrier: yes; RCCL: no)
    virtual bool abort_wakes_peers() const { return false; }
};

// RCCL communicator from a 128-byte ncclUniqueId
int make_rccl_comm(int nranks, int rank, const unsigned char id[128], Comm **out);
// h takes ownership of c (deleted on failure too): sets h->comm, nranks, rank
// and creates the handle's exchange stream and its two events
int attach_comm(lz_handle *h, Comm *c);

}  // namespace lz

// An in-process group of virtual ranks on one device (opaque in the C ABI).
struct lz_local_group;
