// Candidate-batch exchange communicators of libmpcd.so: the collectives the per-step
// exchange uses, behind one interface so mpcd_select / mpcd_mpc_step run the same code on
//  * RcclComm: one process per GPU, RCCL over xGMI (the product path), or
//  * LoopbackComm: N virtual ranks = N contexts on ONE device in one process, each driven by its own
//    host thread, exchanging through device copies ordered by HIP events (single-GPU rehearsal and
//    test of the N-rank logic: rank offsets, gathered-cost order, owner-row sum, flag reduction).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include <string>

enum CommOp { COMM_SUM_F32 = 0, COMM_MAX_I32 = 1 };

struct Comm {
    int nranks = 1, rank = 0;
    virtual ~Comm() {}
    // recv[p * bytes_per_rank ...] = rank p's send (rank order). 0 or an mpcd_status (message in err).
    virtual int allgather(const void *send, void *recv, size_t bytes_per_rank, hipStream_t st, std::string &err) = 0;
    // in place over `count` elements of the op's type
    virtual int allreduce(void *buf, size_t count, CommOp op, hipStream_t st, std::string &err) = 0;
    virtual int broadcast(void *buf, size_t bytes, int root, hipStream_t st, std::string &err) = 0;
};

// RCCL communicator (ncclCommInitRank with a 128-byte unique id shipped out of band).
int comm_create_rccl(int nranks, int rank, const void *id, Comm **out, std::string &err);
int comm_unique_id(void *id_out, std::string &err);
// Virtual rank `rank` of the loopback group `key` (created by its first member, freed with its last).
int comm_create_loopback(int nranks, int rank, uint64_t key, Comm **out, std::string &err);
