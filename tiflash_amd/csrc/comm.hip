// comm.hip — exchange between GPUs (MPP ExchangeSender -> ExchangeReceiver repartition) over RCCL.
//
// Reference: HashPartitionWriter::partitionAndWriteBlocks / MPPTunnelSet::write
// (Flash/Mpp/HashPartitionWriter.cpp:139-204, Flash/Mpp/MPPTunnelSet.cpp) ship each partition's
// encoded packet to the receiver task of that partition over gRPC; ExchangeReceiver
// (Flash/Mpp/ExchangeReceiver.cpp:626-945) decodes them.  Inside one node the MI355X form is one
// process per GPU and one RCCL all-to-all over xGMI per exchanged column: the partition-major
// columns produced by tfg_hash_partition are already the send buffers (partition p = rows
// [offsets[p], offsets[p+1])), so no encode/decode step exists on the device path.
//
// tfg_alltoallv is ncclGroupStart + per-peer ncclSend/ncclRecv + ncclGroupEnd on the context's
// stream (RCCL picks xGMI peer links; one call moves every column byte of one exchange).
#include <vector>
#include <rccl/rccl.h>

#include "common.h"

struct tfg_comm {
    tfg::Ctx *ctx = nullptr;
    ncclComm_t comm = nullptr;
    int nranks = 0;
    int rank = 0;
};

namespace {

int nccl_fail(ncclResult_t r, const char *what) {
    return tfg::fail(TFG_ERR_HIP, "%s: %s", what, ncclGetErrorString(r));
}

#define TFG_NCCL(call)                                                                                          \
    do {                                                                                                        \
        ncclResult_t _r = (call);                                                                               \
        if (_r != ncclSuccess) return nccl_fail(_r, #call);                                                     \
    } while (0)

} // namespace

using namespace tfg;

namespace {

// String end offsets received from several ranks, each relative to its rank's chars: rows
// [start[p], start[p+1]) get add[p] (the chars bytes of the ranks before p)
constexpr int RB_MAX = 64;
struct Rebase {
    uint64_t start[RB_MAX + 1];
    uint64_t add[RB_MAX];
    int n;
};
__global__ void rebase_offsets_kernel(uint64_t *off, Rebase r) {
    const uint64_t total = r.start[r.n];
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (uint64_t)gridDim.x * blockDim.x) {
        int p = 0;
        while (p + 1 < r.n && r.start[p + 1] <= i) ++p;
        off[i] += r.add[p];
    }
}

} // namespace

extern "C" {

int tfg_string_rebase_offsets(tfg_ctx *ctx, uint64_t *offsets, int nparts, const uint64_t *row_start,
                              const uint64_t *add) {
    TFG_CHECK(ctx && nparts >= 1 && row_start && add && (offsets || row_start[nparts] == 0), TFG_ERR_INVALID_ARG,
              "null argument");
    if (int rc = set_device(ctx)) return rc;
    for (int p0 = 0; p0 < nparts; p0 += RB_MAX) {
        Rebase r{};
        r.n = std::min(RB_MAX, nparts - p0);
        for (int p = 0; p <= r.n; ++p) r.start[p] = row_start[p0 + p] - row_start[p0];
        for (int p = 0; p < r.n; ++p) r.add[p] = add[p0 + p];
        const uint64_t rows = r.start[r.n];
        if (!rows) continue;
        hipLaunchKernelGGL(rebase_offsets_kernel, dim3(stream_grid((int64_t)rows, 256, 4096)), dim3(256), 0, ctx->stream,
                           offsets + row_start[p0], r);
        TFG_LAUNCH_CHECK();
    }
    return TFG_OK;
}

int tfg_comm_unique_id(uint8_t *out_id, size_t len) {
    TFG_CHECK(out_id && len >= sizeof(ncclUniqueId), TFG_ERR_INVALID_ARG, "id buffer must hold %zu bytes",
              sizeof(ncclUniqueId));
    ncclUniqueId id;
    TFG_NCCL(ncclGetUniqueId(&id));
    memcpy(out_id, &id, sizeof(id));
    return TFG_OK;
}

int tfg_comm_init(tfg_ctx *ctx, int nranks, int rank, const uint8_t *id, size_t len, tfg_comm **out) {
    TFG_CHECK(ctx && id && out && len >= sizeof(ncclUniqueId), TFG_ERR_INVALID_ARG, "null argument");
    TFG_CHECK(nranks >= 1 && rank >= 0 && rank < nranks, TFG_ERR_INVALID_ARG, "rank %d of %d", rank, nranks);
    if (int rc = set_device(ctx)) return rc;
    ncclUniqueId uid;
    memcpy(&uid, id, sizeof(uid));
    tfg_comm *c = new tfg_comm();
    c->ctx = ctx;
    c->nranks = nranks;
    c->rank = rank;
    ncclResult_t r = ncclCommInitRank(&c->comm, nranks, uid, rank);
    if (r != ncclSuccess) {
        delete c;
        return nccl_fail(r, "ncclCommInitRank");
    }
    *out = c;
    return TFG_OK;
}

int tfg_comm_destroy(tfg_comm *c) {
    if (!c) return TFG_OK;
    if (c->comm) (void)ncclCommDestroy(c->comm);
    delete c;
    return TFG_OK;
}

// Exchange of per-destination byte counts: recv_bytes[p] = what rank p sends to this rank.
int tfg_alltoall_counts(tfg_comm *c, const uint64_t *send_bytes_host, uint64_t *recv_bytes_host) {
    TFG_CHECK(c && send_bytes_host && recv_bytes_host, TFG_ERR_INVALID_ARG, "null argument");
    Ctx *ctx = c->ctx;
    if (int rc = set_device(ctx)) return rc;
    const int P = c->nranks;
    uint64_t *dev = nullptr;
    if (int rc = scratch_get(ctx, (size_t)2 * P * 8, (void **)&dev)) return rc;
    TFG_HIP(hipMemcpyAsync(dev, send_bytes_host, (size_t)P * 8, hipMemcpyHostToDevice, ctx->stream));
    TFG_NCCL(ncclGroupStart());
    for (int p = 0; p < P; ++p) {
        TFG_NCCL(ncclSend(dev + p, 1, ncclUint64, p, c->comm, ctx->stream));
        TFG_NCCL(ncclRecv(dev + P + p, 1, ncclUint64, p, c->comm, ctx->stream));
    }
    TFG_NCCL(ncclGroupEnd());
    TFG_HIP(hipMemcpyAsync(recv_bytes_host, dev + P, (size_t)P * 8, hipMemcpyDeviceToHost, ctx->stream));
    TFG_HIP(hipStreamSynchronize(ctx->stream));
    return TFG_OK;
}

// Variable all-to-all of one byte buffer: the slice [send_displs[p], +send_bytes[p]) goes to rank
// p, rank p's slice lands at [recv_displs[p], +recv_bytes[p]).  Host arrays of nranks entries.
int tfg_alltoallv(tfg_comm *c, const void *send, const uint64_t *send_bytes, const uint64_t *send_displs, void *recv,
                  const uint64_t *recv_bytes, const uint64_t *recv_displs) {
    TFG_CHECK(c && send_bytes && send_displs && recv_bytes && recv_displs, TFG_ERR_INVALID_ARG, "null argument");
    Ctx *ctx = c->ctx;
    if (int rc = set_device(ctx)) return rc;
    TFG_NCCL(ncclGroupStart());
    for (int p = 0; p < c->nranks; ++p) {
        if (send_bytes[p])
            TFG_NCCL(ncclSend((const char *)send + send_displs[p], send_bytes[p], ncclChar, p, c->comm, ctx->stream));
        if (recv_bytes[p])
            TFG_NCCL(ncclRecv((char *)recv + recv_displs[p], recv_bytes[p], ncclChar, p, c->comm, ctx->stream));
    }
    TFG_NCCL(ncclGroupEnd());
    return TFG_OK;
}

// Zero-copy exchange: one RCCL group, a send per (peer, slice) straight from the sender's column
// and a receive per (peer, slice) straight into the receiver's column.  RCCL matches the k-th send
// to a peer with that peer's k-th receive from this rank, so both sides list slices per peer in
// the same order; empty slices are skipped on both sides (the counts exchange told both).
int tfg_exchange_slices(tfg_comm *c, int nsend, const tfg_slice *send, int nrecv, const tfg_slice *recv) {
    TFG_CHECK(c && nsend >= 0 && nrecv >= 0 && (send || !nsend) && (recv || !nrecv), TFG_ERR_INVALID_ARG,
              "null argument");
    Ctx *ctx = c->ctx;
    if (int rc = set_device(ctx)) return rc;
    for (int i = 0; i < nsend; ++i)
        TFG_CHECK(send[i].peer >= 0 && send[i].peer < c->nranks && (send[i].ptr || !send[i].bytes), TFG_ERR_INVALID_ARG,
                  "send slice %d: peer %d, %llu bytes", i, send[i].peer, (unsigned long long)send[i].bytes);
    for (int i = 0; i < nrecv; ++i)
        TFG_CHECK(recv[i].peer >= 0 && recv[i].peer < c->nranks && (recv[i].ptr || !recv[i].bytes), TFG_ERR_INVALID_ARG,
                  "recv slice %d: peer %d, %llu bytes", i, recv[i].peer, (unsigned long long)recv[i].bytes);
    TFG_NCCL(ncclGroupStart());
    for (int i = 0; i < nsend; ++i)
        if (send[i].bytes)
            TFG_NCCL(ncclSend(send[i].ptr, send[i].bytes, ncclChar, send[i].peer, c->comm, ctx->stream));
    for (int i = 0; i < nrecv; ++i)
        if (recv[i].bytes) TFG_NCCL(ncclRecv(recv[i].ptr, recv[i].bytes, ncclChar, recv[i].peer, c->comm, ctx->stream));
    TFG_NCCL(ncclGroupEnd());
    return TFG_OK;
}

// k counts per rank pair: recv[p * k + i] = send[rank * k + i] of rank p
int tfg_alltoall_counts_n(tfg_comm *c, int k, const uint64_t *send_host, uint64_t *recv_host) {
    TFG_CHECK(c && k >= 1 && send_host && recv_host, TFG_ERR_INVALID_ARG, "null argument");
    Ctx *ctx = c->ctx;
    if (int rc = set_device(ctx)) return rc;
    const int P = c->nranks;
    uint64_t *dev = nullptr;
    if (int rc = scratch_get(ctx, (size_t)2 * P * k * 8, (void **)&dev)) return rc;
    TFG_HIP(hipMemcpyAsync(dev, send_host, (size_t)P * k * 8, hipMemcpyHostToDevice, ctx->stream));
    TFG_NCCL(ncclGroupStart());
    for (int p = 0; p < P; ++p) {
        TFG_NCCL(ncclSend(dev + (size_t)p * k, (size_t)k, ncclUint64, p, c->comm, ctx->stream));
        TFG_NCCL(ncclRecv(dev + (size_t)(P + p) * k, (size_t)k, ncclUint64, p, c->comm, ctx->stream));
    }
    TFG_NCCL(ncclGroupEnd());
    TFG_HIP(hipMemcpyAsync(recv_host, dev + (size_t)P * k, (size_t)P * k * 8, hipMemcpyDeviceToHost, ctx->stream));
    TFG_HIP(hipStreamSynchronize(ctx->stream));
    return TFG_OK;
}

int tfg_comm_info(tfg_comm *c, int *nranks, int *rank) {
    TFG_CHECK(c, TFG_ERR_INVALID_ARG, "null argument");
    if (nranks) *nranks = c->nranks;
    if (rank) *rank = c->rank;
    return TFG_OK;
}

} // extern "C"
