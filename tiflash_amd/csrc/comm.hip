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

// Batched copy: up to CP_MAX {src, dst, bytes} descriptors per launch (src null = zero fill),
// passed by value; workgroup w copies 64 KB chunk w of the flattened descriptors, 16 bytes a lane
// where both ends are 16-byte aligned, 8 / 1 bytes otherwise.
constexpr int CP_MAX = 120; // the descriptor block stays under 4 KB of kernel arguments
constexpr uint64_t CP_CHUNK = 64 * 1024;
struct CopyDescs {
    const uint8_t *src[CP_MAX];
    uint8_t *dst[CP_MAX];
    uint64_t bytes[CP_MAX];
    uint64_t first_chunk[CP_MAX + 1]; // exclusive prefix of each descriptor's chunk count
    int n;
};

__global__ void __launch_bounds__(256) batched_copy_kernel(CopyDescs d) {
    const uint64_t c = blockIdx.x;
    int lo = 0, hi = d.n - 1; // the descriptor of chunk c: the last with first_chunk <= c
    while (lo < hi) {
        const int mid = (lo + hi + 1) / 2;
        if (d.first_chunk[mid] <= c) lo = mid;
        else hi = mid - 1;
    }
    const uint64_t off = (c - d.first_chunk[lo]) * CP_CHUNK;
    const uint64_t len = d.bytes[lo] - off < CP_CHUNK ? d.bytes[lo] - off : CP_CHUNK;
    const uint8_t *s = d.src[lo] ? d.src[lo] + off : nullptr;
    uint8_t *t = d.dst[lo] + off;
    const uintptr_t al = (uintptr_t)t | (s ? (uintptr_t)s : 0);
    if ((al & 15) == 0) {
        for (uint64_t i = threadIdx.x * 16; i + 16 <= len; i += 256 * 16)
            *(uint4 *)(t + i) = s ? *(const uint4 *)(s + i) : make_uint4(0, 0, 0, 0);
        for (uint64_t i = (len & ~(uint64_t)15) + threadIdx.x; i < len; i += 256) t[i] = s ? s[i] : 0;
    } else if ((al & 7) == 0) {
        for (uint64_t i = threadIdx.x * 8; i + 8 <= len; i += 256 * 8)
            *(uint64_t *)(t + i) = s ? *(const uint64_t *)(s + i) : 0ull;
        for (uint64_t i = (len & ~(uint64_t)7) + threadIdx.x; i < len; i += 256) t[i] = s ? s[i] : 0;
    } else {
        for (uint64_t i = threadIdx.x; i < len; i += 256) t[i] = s ? s[i] : 0;
    }
}

struct CopyBatch {
    Ctx *ctx;
    CopyDescs d{};
    uint64_t chunks = 0;
    int add(const void *src, void *dst, uint64_t bytes) {
        if (!bytes) return TFG_OK;
        if (d.n == CP_MAX)
            if (int rc = flush()) return rc;
        d.src[d.n] = (const uint8_t *)src;
        d.dst[d.n] = (uint8_t *)dst;
        d.bytes[d.n] = bytes;
        d.first_chunk[d.n] = chunks;
        chunks += (bytes + CP_CHUNK - 1) / CP_CHUNK;
        ++d.n;
        return TFG_OK;
    }
    int flush() {
        if (!d.n) return TFG_OK;
        d.first_chunk[d.n] = chunks;
        hipLaunchKernelGGL(batched_copy_kernel, dim3((unsigned)chunks), dim3(256), 0, ctx->stream, d);
        TFG_LAUNCH_CHECK();
        d.n = 0;
        chunks = 0;
        return TFG_OK;
    }
};

} // namespace

extern "C" {

int tfg_pack_planes(tfg_ctx *ctx, int nparts, int nplanes, const void *const *planes, const int *widths,
                    const uint64_t *rows, void *out, uint64_t *out_seg_bytes) {
    TFG_CHECK(ctx && widths && rows && out_seg_bytes && nparts >= 1 && nplanes >= 1 && (planes || nplanes == 0),
              TFG_ERR_INVALID_ARG, "null argument");
    if (int rc = set_device(ctx)) return rc;
    CopyBatch cb{ctx};
    uint64_t o = 0;
    for (int p = 0; p < nparts; ++p) {
        const uint64_t s0 = o;
        for (int j = 0; j < nplanes; ++j) {
            TFG_CHECK(widths[j] > 0, TFG_ERR_INVALID_ARG, "plane %d width %d", j, widths[j]);
            const uint64_t b = rows[(size_t)p * nplanes + j] * (uint64_t)widths[j];
            TFG_CHECK(!b || out, TFG_ERR_INVALID_ARG, "null output");
            if (int rc = cb.add(planes[(size_t)p * nplanes + j], (uint8_t *)out + o, b)) return rc;
            o += b;
        }
        out_seg_bytes[p] = o - s0;
    }
    return cb.flush();
}

int tfg_unpack_planes(tfg_ctx *ctx, int nparts, int nplanes, const int *widths, const uint64_t *rows, const void *in,
                      void *const *planes) {
    TFG_CHECK(ctx && widths && rows && planes && nparts >= 1 && nplanes >= 1, TFG_ERR_INVALID_ARG, "null argument");
    if (int rc = set_device(ctx)) return rc;
    CopyBatch cb{ctx};
    std::vector<uint64_t> r0(nplanes, 0); // rows of plane j already placed
    uint64_t o = 0;
    for (int p = 0; p < nparts; ++p) {
        for (int j = 0; j < nplanes; ++j) {
            TFG_CHECK(widths[j] > 0, TFG_ERR_INVALID_ARG, "plane %d width %d", j, widths[j]);
            const uint64_t r = rows[(size_t)p * nplanes + j], b = r * (uint64_t)widths[j];
            TFG_CHECK(!b || (in && planes[j]), TFG_ERR_INVALID_ARG, "null buffer");
            if (int rc = cb.add((const uint8_t *)in + o, (uint8_t *)planes[j] + r0[j] * widths[j], b)) return rc;
            o += b;
            r0[j] += r;
        }
    }
    return cb.flush();
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

int tfg_comm_info(tfg_comm *c, int *nranks, int *rank) {
    TFG_CHECK(c, TFG_ERR_INVALID_ARG, "null argument");
    if (nranks) *nranks = c->nranks;
    if (rank) *rank = c->rank;
    return TFG_OK;
}

} // extern "C"
