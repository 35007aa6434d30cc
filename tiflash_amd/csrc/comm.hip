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

extern "C" {

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

int tfg_comm_info(tfg_comm *c, int *nranks, int *rank) {
    TFG_CHECK(c, TFG_ERR_INVALID_ARG, "null argument");
    if (nranks) *nranks = c->nranks;
    if (rank) *rank = c->rank;
    return TFG_OK;
}

} // extern "C"
