// tfa_host.h — C++ host operators above the C-ABI (include/tiflash_amd.h).
//
// The reference's drop-in surface for this path is C++: FilterTransformAction,
// the Aggregator facade, the Join facade, HashPartitionWriter and the IBlockInputStream wrappers
// that PhysicalPlan instantiates from tipb::Executor.  This layer restates those interfaces over
// device-resident columns — same names, argument meaning and error behaviour — and calls only
// the C-ABI (no HIP, no torch).  Differences from the reference are listed per class.
//
//   Block / ColumnWithTypeAndName      Core/Block.h:41, Core/ColumnWithTypeAndName.h
//   IColumn (immutable, COW-shared)    Columns/IColumn.h:426 (filter returns a new column)
//   DB::Exception + ErrorCodes         Common/Exception.h, Common/ErrorCodes.cpp:30-198
//   ExpressionActions                  Interpreters/ExpressionActions.cpp:351-364,547
//   FilterTransformAction              DataStreams/FilterTransformAction.cpp:32-173
//   Aggregator (Params, executeOnBlock, merge, convertToBlocks)  Interpreters/Aggregator.h:855-1035
//   Join (initBuild, insertFromBlock, finishOneBuild, joinBlock)  Interpreters/Join.h:191-283
//   HashPartitionWriter (write, flush)  Flash/Mpp/HashPartitionWriter.cpp:76-204
//   IBlockInputStream (getHeader, read) DataStreams/IBlockInputStream.h:60-201
#pragma once

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <functional>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/tiflash_amd.h"

namespace tfa {

// ---------------------------------------------------------------- errors (Common/ErrorCodes.cpp)
namespace ErrorCodes {
constexpr int SIZES_OF_COLUMNS_DOESNT_MATCH = 9;
constexpr int BAD_ARGUMENTS = 36;
constexpr int ILLEGAL_TYPE_OF_ARGUMENT = 43;
constexpr int NOT_IMPLEMENTED = 48;
constexpr int LOGICAL_ERROR = 49;
constexpr int ILLEGAL_TYPE_OF_COLUMN_FOR_FILTER = 59;
constexpr int CANNOT_ALLOCATE_MEMORY = 173;
constexpr int NOT_FOUND_COLUMN_IN_BLOCK = 10;
constexpr int DECIMAL_OVERFLOW = 446;
} // namespace ErrorCodes

class Exception : public std::runtime_error {
public:
    Exception(const std::string &msg, int code) : std::runtime_error(msg), code_(code) {}
    int code() const { return code_; }

private:
    int code_;
};

// Maps a tfg status to the reference's error code and throws (no-op on TFG_OK).
void check(int status, const char *what);

// ---------------------------------------------------------------- device context
class Context {
public:
    explicit Context(int device = 0);
    ~Context();
    Context(const Context &) = delete;
    Context &operator=(const Context &) = delete;
    tfg_ctx *raw() const { return ctx_; }
    void sync() const;
    int device() const { return device_; }

private:
    tfg_ctx *ctx_ = nullptr;
    int device_ = 0;
};

// device allocation owned by a column (freed with the last reference)
class DeviceBuffer {
public:
    DeviceBuffer(Context &ctx, size_t bytes);
    ~DeviceBuffer();
    DeviceBuffer(const DeviceBuffer &) = delete;
    DeviceBuffer &operator=(const DeviceBuffer &) = delete;
    void *data() const { return ptr_; }
    size_t bytes() const { return bytes_; }

private:
    Context &ctx_;
    void *ptr_ = nullptr;
    size_t bytes_ = 0;
};
using DeviceBufferPtr = std::shared_ptr<DeviceBuffer>;

// ---------------------------------------------------------------- types and columns
// DataTypeDecimal carries (precision, scale) (DataTypes/DataTypeDecimal.h); prec 0 means the
// storage type's maximum (Decimal32 9, Decimal64 18, Decimal128 38, Decimal256 65).
struct DataType {
    int type = TFG_INT64; // tfg_type, or TYPE_STRING
    int scale = 0;        // Decimal scale
    int prec = 0;         // Decimal precision (0 = the storage type's maximum)
    bool nullable = false;
    static constexpr int TYPE_STRING = 100;
    size_t width() const; // bytes per value (0 for String)
    bool isString() const { return type == TYPE_STRING; }
    bool isDecimal() const {
        return type == TFG_DECIMAL32 || type == TFG_DECIMAL64 || type == TFG_DECIMAL128 || type == TFG_DECIMAL256;
    }
    int precision() const; // prec, or the storage type's maximum
    std::string getName() const;
    bool operator==(const DataType &o) const {
        return type == o.type && scale == o.scale && nullable == o.nullable && (!isDecimal() || precision() == o.precision());
    }
    // createDecimal(prec, scale): the narrowest storage type of a precision (DataTypes/DataTypeDecimal.h)
    static DataType decimal(int prec, int scale, bool nullable = false);
};

// Immutable device column: fixed-width values (`data`), or String chars + UInt64 end offsets
// (ColumnString layout, each row '\0'-terminated); optional NULL map (ColumnNullable).  A
// const column (ColumnConst) keeps one host value and a row count.
struct IColumn {
    DataType type;
    size_t rows = 0;
    DeviceBufferPtr data;    // values, or chars for String
    DeviceBufferPtr offsets; // String only: rows x UInt64
    DeviceBufferPtr nullmap; // rows x UInt8 (1 = NULL) or null
    size_t chars = 0;        // String only: bytes in `data`
    bool is_const = false;
    uint64_t const_value = 0; // is_const: the bits of the one value

    size_t size() const { return rows; }
    bool isColumnConst() const { return is_const; }
    const void *dataPtr() const { return data ? data->data() : nullptr; }
    const uint8_t *nullPtr() const { return nullmap ? (const uint8_t *)nullmap->data() : nullptr; }
};
using ColumnPtr = std::shared_ptr<const IColumn>;

struct ColumnWithTypeAndName {
    ColumnPtr column;
    DataType type;
    std::string name;
};

// BlockInfo (Core/BlockInfo.h:25-57): bucket_num of a two-level bucket, and the selective row
// list — when set, only the rows it lists take part (weak hash + scatter of the exchange,
// HashBaseWriterHelper.cpp:110-260); produced by auto pass-through aggregation.  Here the list
// is a device array of UInt64 row ids.
struct BlockSelective {
    DeviceBufferPtr rows; // count x UInt64 row ids (device)
    size_t count = 0;
    size_t size() const { return count; }
    const uint64_t *data() const { return rows ? (const uint64_t *)rows->data() : nullptr; }
};
using BlockSelectivePtr = std::shared_ptr<BlockSelective>;
BlockSelectivePtr makeSelective(Context &ctx, const std::vector<uint64_t> &rows);

struct BlockInfo {
    int32_t bucket_num = -1;
    BlockSelectivePtr selective;
};

class Block {
public:
    Block() = default;
    Block(std::initializer_list<ColumnWithTypeAndName> cols) : data_(cols) {}
    explicit Block(std::vector<ColumnWithTypeAndName> cols) : data_(std::move(cols)) {}
    void insert(ColumnWithTypeAndName c) { data_.push_back(std::move(c)); }
    void insert(size_t position, ColumnWithTypeAndName c);
    void erase(size_t position);
    size_t columns() const { return data_.size(); }
    size_t rows() const; // checks every column has the same size
    bool has(const std::string &name) const;
    size_t getPositionByName(const std::string &name) const;
    const ColumnWithTypeAndName &getByName(const std::string &name) const;
    ColumnWithTypeAndName &safeGetByPosition(size_t i);
    const ColumnWithTypeAndName &safeGetByPosition(size_t i) const;
    Block cloneEmpty() const;
    void clear() { data_.clear(); }
    explicit operator bool() const { return !data_.empty(); }
    const std::vector<ColumnWithTypeAndName> &getColumnsWithTypeAndName() const { return data_; }
    BlockInfo info;

private:
    std::vector<ColumnWithTypeAndName> data_;
};

// host <-> device helpers (tests, sources, sinks)
ColumnPtr makeColumn(Context &ctx, DataType type, const void *values, size_t rows,
                     const uint8_t *nullmap = nullptr);
ColumnPtr makeStringColumn(Context &ctx, const std::vector<std::string> &values,
                           const uint8_t *nullmap = nullptr);
ColumnPtr makeConstColumn(DataType type, uint64_t bits, size_t rows);
ColumnPtr materialize(Context &ctx, const ColumnPtr &c); // ColumnConst -> full column
std::vector<uint8_t> toHostBytes(Context &ctx, const IColumn &c);
std::vector<uint8_t> toHostNullMap(Context &ctx, const IColumn &c);
std::vector<std::string> toHostStrings(Context &ctx, const IColumn &c);
template <typename T> std::vector<T> toHost(Context &ctx, const IColumn &c) {
    std::vector<uint8_t> b = toHostBytes(ctx, c);
    std::vector<T> out(c.rows);
    if (!b.empty()) memcpy(out.data(), b.data(), std::min(b.size(), out.size() * sizeof(T)));
    return out;
}
// Concatenates blocks with the same structure (Join build side, partition buffers).
Block concatenateBlocks(Context &ctx, const std::vector<Block> &blocks);
// Rows of `src` at `perm` (0xFFFFFFFF -> default value and, when make_nullable, NULL).
ColumnPtr gatherColumn(Context &ctx, const IColumn &src, const uint32_t *perm_dev, size_t n, bool make_nullable);

// ---------------------------------------------------------------- expressions (a1-a4)
// A literal (Field) for constant operands.
struct Field {
    int type = TFG_INT64;
    uint64_t bits = 0;
    static Field Int64(int64_t v);
    static Field UInt64(uint64_t v);
    static Field Float64(double v);
    static Field Decimal64(int64_t raw, int scale);
    int scale = 0;
    int prec = 0; // Decimal literal precision (0 = the storage type's maximum)
};

// ExpressionActions restricted to the functions on the hot path: comparisons, and/or/not,
// plus/minus/multiply.  execute(block) appends each action's result column like the
// reference's ExpressionActions::execute (Interpreters/ExpressionActions.cpp:351-364).
class ExpressionActions {
public:
    explicit ExpressionActions(Context &ctx) : ctx_(ctx) {}
    // result = lhs Op constant   (equals/notEquals/less/greater/lessOrEquals/greaterOrEquals)
    ExpressionActions &compare(const std::string &lhs, int op, Field constant, const std::string &result);
    // result = lhs Op rhs (columns)
    ExpressionActions &compareColumns(const std::string &lhs, int op, const std::string &rhs, const std::string &result);
    // result = and/or(a, b) or not(a)
    ExpressionActions &logical(int op, const std::string &a, const std::string &b, const std::string &result);
    // result = a (+|-|*) b; b may be a constant; result type / scale as FunctionBinaryArithmetic infers
    ExpressionActions &arithmetic(int op, const std::string &a, const std::string &b, const std::string &result);
    ExpressionActions &arithmeticConst(int op, const std::string &a, Field b, const std::string &result);
    // result = constant (+|-|*) b
    ExpressionActions &arithmeticConstLeft(int op, Field a, const std::string &b, const std::string &result);
    void execute(Block &block) const;
    // the fused form: a single `column Op constant` predicate feeding a filter / aggregation
    bool singleCompare(std::string &column, int &op, Field &constant, std::string &result) const;

private:
    struct Action {
        int kind; // 0 compare-const, 1 compare-cols, 2 logical, 3 arith, 4 arith-const, 5 const-arith
        int op;
        std::string a, b, result;
        Field constant;
    };
    Context &ctx_;
    std::vector<Action> actions_;
};
using ExpressionActionsPtr = std::shared_ptr<ExpressionActions>;

// ---------------------------------------------------------------- filter (a5-a8)
using FilterPtr = ColumnPtr; // UInt8 mask column

class FilterTransformAction {
public:
    FilterTransformAction(Context &ctx, const Block &header, ExpressionActionsPtr expression,
                          const std::string &filter_column_name);
    // Same contract as the reference (:72-173): returns false if every row is filtered out
    // (block untouched), true otherwise; with return_filter the mask is returned instead of
    // filtering (nullptr when all rows pass).  The filter column becomes a constant 1.
    bool transform(Block &block, FilterPtr &res_filter, bool return_filter);
    Block getHeader() const { return header_; }

private:
    Context &ctx_;
    Block header_;
    ExpressionActionsPtr expression_;
    std::string filter_column_name_;
};

// ---------------------------------------------------------------- aggregation (a9-a17)
struct AggregateDescription {
    std::string function;                    // "sum" | "count" | "min" | "max" | "first_row"
    std::vector<std::string> argument_names; // count() has none
    std::string column_name;
    // min / max over a String: the collator the comparisons use (IAggregateFunction::setCollators,
    // SingleValueDataString::setCollators, AggregateFunctionMinMaxAny.h:272-275)
    int collator = TFG_COLLATOR_NONE;
};
using AggregateDescriptions = std::vector<AggregateDescription>;

class Aggregator {
public:
    struct Params {
        Block src_header;
        // 0 or 1 fixed-width key (key8..key64 / nullable), or several fixed keys of <= 16 bytes
        // (keys128 / nullable_keys128) or one String key (key_string, sort key <= 15 bytes)
        std::vector<std::string> keys;
        AggregateDescriptions aggregates;
        std::vector<int> collators; // tfg_collator of a String key (empty = binary)
        int bucket_bits = 0;
        int64_t expected_groups = 0;
    };
    Aggregator(Context &ctx, const Params &params);
    ~Aggregator();
    Aggregator(const Aggregator &) = delete;
    Aggregator &operator=(const Aggregator &) = delete;
    // executeOnBlock (Aggregator.cpp:1127-1246); `filter` (optional UInt8 mask) skips rows
    void executeOnBlock(const Block &block, const FilterPtr &filter = nullptr);
    // fused FilterTransformAction -> Aggregator for `pred Op constant`
    void executeOnBlockFiltered(const Block &block, const std::string &pred, int op, Field constant);
    // two-phase final aggregation: a Block of (key, partial states) from convertToBlock(false)
    void mergeOnBlock(const Block &partial);
    void merge(Aggregator &other); // mergeDataImpl of two variants with one signature
    size_t size() const;
    // final = true: result columns (sum of nullable args is NULL when it saw no value);
    // final = false: partial states (key, sum / count state columns) for an exchange
    Block convertToBlock(bool final = true) const;
    void reset();
    tfg_agg *raw() const { return agg_; }

private:
    Context &ctx_;
    Params params_;
    tfg_agg *agg_ = nullptr;
    DataType key_type_;
    std::vector<DataType> key_types_; // every key (packed methods)
    bool packed_ = false;             // keys128 / key_string through tfg_agg_*_keys
    std::vector<int> kinds_;          // device aggregates (tfg_agg_kind)
    std::vector<DataType> arg_types_; // ... and their argument types
    // aggregate i -> its device aggregate, or -1 for first_row of a GROUP BY column, which is the
    // key itself (agg_func_ref_key: AggKeyOptimization, gtest_aggregation_executor.cpp:1053-1137)
    std::vector<int> dev_index_;
    std::vector<int> ref_key_; // aggregate i -> the key index it repeats (-1: none)
    bool hidden_count_ = false; // every aggregate repeats a key: the device aggregator counts rows
    // String arguments / states travel as tfg_str_col structs held in `strs`
    void argPointers(const Block &b, std::vector<const void *> &args, std::vector<const uint8_t *> &nulls,
                     std::vector<ColumnPtr> &hold, std::vector<std::unique_ptr<tfg_str_col>> &strs) const;
    void insertAggregateColumns(Block &out, const std::vector<std::shared_ptr<IColumn>> &states,
                                const std::vector<ColumnPtr> &keys, size_t g) const;
    void keyPointers(const Block &b, std::vector<const void *> &cols, std::vector<const uint64_t *> &offs,
                     std::vector<const uint8_t *> &nulls, std::vector<ColumnPtr> &hold) const;
};

// ---------------------------------------------------------------- hash join (a18-a21)
// Inner / Left / Semi / Anti map onto tfg_join_kind; LeftOuterSemi / AntiLeftOuterSemi (tipb
// TypeLeftOuterSemiJoin / TypeAntiLeftOuterSemiJoin) return every probe row plus a Nullable(Int8)
// match column and are derived on the host from an INNER probe + tfg_join_mark.
enum class JoinKind {
    Inner = TFG_JOIN_INNER,
    Left = TFG_JOIN_LEFT,
    Semi = TFG_JOIN_SEMI,
    Anti = TFG_JOIN_ANTI,
    LeftOuterSemi = 100,
    AntiLeftOuterSemi = 101
};

class Join {
public:
    Join(Context &ctx, JoinKind kind, const std::string &probe_key, const std::string &build_key,
         int64_t expected_build_rows = 0);
    // Several key columns, or String / 16-byte / float keys (chooseJoinMapMethod keys128 /
    // keys256 / key_strbin / key_strbinpadding / serialized, JoinHashMap.cpp:33-116): joined on
    // device fingerprints of the key tuples, every candidate pair verified on the full keys.
    // collators[j] (tfg_collator) applies to String key j; empty = binary.
    Join(Context &ctx, JoinKind kind, std::vector<std::string> probe_keys, std::vector<std::string> build_keys,
         int64_t expected_build_rows = 0, std::vector<int> collators = {});
    ~Join();
    Join(const Join &) = delete;
    Join &operator=(const Join &) = delete;
    void initBuild(const Block &sample_block);
    void insertFromBlock(const Block &block); // rows with a NULL key are not inserted
    void finishOneBuild();
    // probe columns replicated per match, then the build block's non-key columns (LEFT: NULL
    // where unmatched).  SEMI / ANTI return the probe columns of the qualifying rows.
    Block joinBlock(const Block &probe_block);
    uint64_t buildRows() const;
    // JoinNonEqualConditions::other_cond_expr / other_cond_name (Interpreters/Join.cpp:798-1150):
    // evaluated over the joined (probe + build) columns of every key-equal pair; NULL = false.
    void setOtherCondition(ExpressionActionsPtr expr, std::string filter_column);
    // LeftOuterSemi / AntiLeftOuterSemi: name of the match column (default "match_helper")
    void setMatchHelperName(std::string name) { match_helper_ = std::move(name); }
    // JoinV2 (HashJoinPointerTable): build into a pointer table (tagged heads when `tagged`)
    // instead of radix partitions; call before the first insertFromBlock
    void useJoinV2(bool tagged = true) { v2_flags_ = tagged ? TFG_JOIN_V2_TAGGED : 0; }

private:
    Context &ctx_;
    JoinKind kind_;
    std::vector<std::string> probe_keys_, build_keys_;
    std::vector<int> collators_;
    bool general_keys_ = false; // fingerprint + verify (several / String / wide keys)
    int64_t expected_;
    tfg_join *join_ = nullptr;
    Block sample_;
    std::vector<Block> build_blocks_;
    Block build_; // concatenated at finishOneBuild
    bool finished_ = false;
    ExpressionActionsPtr other_cond_;
    std::string other_filter_;
    std::string match_helper_ = "match_helper";
    int v2_flags_ = -1; // >= 0: JoinV2 pointer table
    Block joinBlockWithCondition(const Block &probe_block);
    ColumnPtr joinKey(const Block &block, const std::vector<std::string> &names) const;
    DeviceBufferPtr verifyKeys(const Block &probe_block, const uint32_t *pi, const uint32_t *bi, uint64_t count,
                               DeviceBufferPtr pass) const;
};

// ---------------------------------------------------------------- exchange (a22-a24, e)
// HashPartitionWriter::write / flush (HashPartitionWriter.cpp:76-204): rows are buffered until
// batch_send_min_limit, then weak-hashed on the partition key columns, routed with fillSelector
// (part = (h * P) >> 32) and scattered stably; `sink(part, block)` receives each partition's
// block (the ExchangeSender tunnel; with an MPPExchange it is an all-to-all).
class HashPartitionWriter {
public:
    using Sink = std::function<void(uint32_t, Block &&)>;
    HashPartitionWriter(Context &ctx, std::vector<size_t> partition_col_ids, uint32_t partition_num, Sink sink,
                        int64_t batch_send_min_limit = -1);
    void write(const Block &block);
    void flush();
    // collators of the partition key columns (String keys; TiDB::TiDBCollators in the reference)
    void setCollators(std::vector<int> collators) { collators_ = std::move(collators); }

private:
    Context &ctx_;
    std::vector<size_t> partition_col_ids_;
    uint32_t partition_num_;
    Sink sink_;
    int64_t limit_;
    std::vector<Block> pending_;
    size_t pending_rows_ = 0;
    std::vector<int> collators_;
};

// A device packet (codec output): `bytes` valid bytes of `buf`.
struct DevicePacket {
    DeviceBufferPtr buf;
    size_t bytes = 0;
    bool empty() const { return bytes == 0; }
};

// FineGrainedShuffleWriter (Flash/Mpp/FineGrainedShuffleWriter.cpp; chosen by newMPPExchangeWriter.cpp:66-78
// for a Hash exchange with fine_grained_shuffle_stream_count > 0): rows are routed to
// partition_num * stream_count buckets (fillSelectorForFineGrainedShuffle, HashBaseWriterHelper.cpp:64-84:
// bucket = ((h * P) >> 32) * S + h % S), and each flush sends ONE packet per partition whose chunks
// are that partition's non-empty stream buckets, V1-encoded, tagged with their stream ids
// (MPPTunnelSetHelper::ToFineGrainedPacket).  The receiving side routes chunk i to stream
// stream_ids[i] (ExchangeReceiver's fine-grained queues).
struct FineGrainedPacket {
    std::vector<uint32_t> stream_ids;
    std::vector<DevicePacket> chunks; // CHBlockChunkCodecV1 packets (compression NONE)
};
class FineGrainedShuffleWriter {
public:
    using Sink = std::function<void(uint32_t, FineGrainedPacket &&)>;
    FineGrainedShuffleWriter(Context &ctx, std::vector<size_t> partition_col_ids, uint32_t partition_num,
                             uint32_t stream_count, uint64_t batch_size, Sink sink,
                             uint64_t max_buffered_bytes = (uint64_t)16 << 20);
    void write(const Block &block);
    void flush();
    void setCollators(std::vector<int> collators) { collators_ = std::move(collators); }

private:
    Context &ctx_;
    std::vector<size_t> partition_col_ids_;
    uint32_t partition_num_, stream_count_;
    uint64_t max_buffered_rows_, max_buffered_bytes_;
    Sink sink_;
    std::vector<int> collators_;
    Block header_;
    bool header_set_ = false;
    std::vector<Block> blocks_;
    uint64_t buffered_rows_ = 0, buffered_bytes_ = 0;
};

// Partition a block into partition_num * stream_count fine-grained buckets (bucket p * S + s).
std::vector<Block> fineGrainedPartitionBlock(Context &ctx, const Block &block, const std::vector<size_t> &key_ids,
                                             uint32_t partition_num, uint32_t stream_count,
                                             const std::vector<int> &collators = {});

// Partition a block into partition_num blocks (the scatterColumns step alone).
// String columns (keys hashed by ColumnString::updateWeakHash32 under collators[k], the k-th
// key's collator) are scattered through the stable partition permutation.
std::vector<Block> hashPartitionBlock(Context &ctx, const Block &block, const std::vector<size_t> &key_ids,
                                      uint32_t partition_num, const std::vector<int> &collators = {});

// The collective under an MPP exchange between the ranks of one query (what MPPTunnelSet's
// tunnels carry between tasks): a counts exchange, then the zero-copy exchange of device slices
// (tfg_exchange_slices).  RcclTransport is the product's (tfg_comm: RCCL over xGMI, one process
// per GPU); tests plug in other transports (tests/cpp/test_host.cpp runs two processes over TCP).
class ExchangeTransport {
public:
    virtual ~ExchangeTransport() = default;
    virtual int nranks() const = 0;
    virtual int rank() const = 0;
    // k counts per rank pair: recv[p * k + i] = send[this rank * k + i] of rank p (host arrays)
    virtual void alltoallCountsN(int k, const uint64_t *send, uint64_t *recv) = 0;
    // every send slice to its peer, every receive slice from its peer (device memory in place);
    // a peer's k-th send matches that peer's k-th receive from this rank
    virtual void exchangeSlices(const std::vector<tfg_slice> &send, const std::vector<tfg_slice> &recv) = 0;
};

class RcclTransport : public ExchangeTransport {
public:
    RcclTransport(Context &ctx, int nranks, int rank, const uint8_t *unique_id, size_t id_len);
    ~RcclTransport() override;
    int nranks() const override { return nranks_; }
    int rank() const override { return rank_; }
    void alltoallCountsN(int k, const uint64_t *send, uint64_t *recv) override;
    void exchangeSlices(const std::vector<tfg_slice> &send, const std::vector<tfg_slice> &recv) override;

private:
    tfg_comm *comm_ = nullptr;
    int nranks_, rank_;
};

// One-node exchange: every rank contributes partition_num == nranks blocks and receives the
// concatenation of its partition from every rank (ExchangeReceiver output).  Zero copy: one counts
// exchange, then every column plane's slice goes from the partition block where it lies to the
// output column at its row offset (tfg_exchange_slices: one RCCL group per call, no pack / unpack,
// no packet encode / decode).  String columns travel as their end offsets (rebased on arrival,
// tfg_string_rebase_offsets) and chars; a Nullable column's null map as a plane of its own (a
// partition without one sends nothing and its rows stay zero).
class MPPExchange {
public:
    MPPExchange(Context &ctx, int nranks, int rank, const uint8_t *unique_id, size_t id_len); // over RCCL
    MPPExchange(Context &ctx, std::shared_ptr<ExchangeTransport> transport);
    Block exchange(const std::vector<Block> &partitions);
    int nranks() const { return nranks_; }
    int rank() const { return rank_; }

private:
    Context &ctx_;
    std::shared_ptr<ExchangeTransport> t_;
    int nranks_, rank_;
};

// ---------------------------------------------------------------- auto pass-through (f4)
// AutoPassThroughHashAggContext (Operators/AutoPassThroughHashAggContext.{h,cpp}, design doc
// docs/design/2024-08-07-auto-pass-through-hashagg.md): the first stage of a two-stage
// aggregation decides at run time whether pre-aggregating pays.  Same states, thresholds and
// switching rules: Init (until the hash map passes 2 MB) -> Adjust (insert, measure the hit
// rate over normal_row_limit rows) -> PreHashAgg (hit rate >= 0.9) / PassThrough (<= 0.2) /
// Selective (between: rows whose key is in the map are aggregated, the others pass through)
// -> back to Adjust after normal / dynamic row limits (dynamic doubles up to 100 units).
// Pass-through blocks carry the final-form columns of one row per group
// (AutoPassThroughHashAggHelper.cpp): keys copied, sum(x) widened to the sum type (NULL kept),
// count(x) = 0/1, count() = 1.  Differences: the hash-map byte size is restated from the group
// count (16-byte cells at <= 50% load, as HashMap<UInt64, AggregateDataPtr>); Selective rows
// are materialised (filtered) instead of flagged in Block::info.selective.
class AutoPassThroughHashAggContext {
public:
    enum class State { Init, Adjust, PreHashAgg, PassThrough, Selective };
    static constexpr size_t INIT_STATE_HASHMAP_THRESHOLD = 2 * 1024 * 1024;
    static constexpr size_t MAX_DYNAMIC_UNIT_LIMIT = 100;
    static constexpr double PassThroughRateLimit = 0.2;
    static constexpr double PreHashAggRateLimit = 0.9;

    // spill_threshold_bytes (0 = off): the revocable bytes past which the map is marked for
    // spill after a block (Aggregator::executeOnBlock -> AggSpillContext::
    // updatePerThreadRevocableMemory -> AggregatedDataVariants::tryMarkNeedSpill,
    // Aggregator.cpp:79-92,1236-1243).  Auto pass-through never spills to disk: a map marked for
    // spill is handed over in advance and every later row passes through
    // (AutoPassThroughHashAggContext.cpp:86-104).
    AutoPassThroughHashAggContext(Context &ctx, const Aggregator::Params &params, uint64_t row_limit_unit,
                                  uint64_t normal_unit_num = 1, uint64_t dynamic_unit_num = 5,
                                  size_t spill_threshold_bytes = 0);
    void onBlock(const Block &block, bool force_streaming = false);
    // the map's final block first when it is marked for spill (once), else the next pass-through
    // block, or an empty Block
    Block tryGetDataInAdvance();
    Block getDataFromHashTable(); // the hash map's final block (once; the map is then closed)
    // AggregateContext::needSpill(task, try_mark_need_spill = true): the query's memory policy
    // marks the map (no-op on an empty map, as tryMarkNeedSpill)
    bool tryMarkNeedSpill();
    bool needSpill() const { return need_spill_; }
    // hash map + aggregate states in bytes (AggregatedDataVariants::revocableBytes)
    size_t revocableBytes() const;
    Block getHeader() const { return header_; }
    State state() const { return state_; }
    size_t hashMapBytes() const;
    size_t passThroughRows() const { return pass_through_rows_; }
    size_t aggregatedRows() const { return aggregated_rows_; }

private:
    Context &ctx_;
    Aggregator::Params params_;
    Aggregator agg_;
    Block header_;
    State state_ = State::Init;
    size_t normal_row_limit_, dynamic_row_limit_, row_limit_unit_, max_dynamic_row_limit_;
    size_t adjust_processed_rows_ = 0, adjust_hit_rows_ = 0, state_processed_rows_ = 0;
    size_t pass_through_rows_ = 0, aggregated_rows_ = 0;
    bool already_get_data_from_hash_table_ = false;
    size_t spill_threshold_ = 0;
    bool need_spill_ = false;
    void forceState();
    std::vector<Block> buffer_;
    size_t buffer_head_ = 0;
    std::unique_ptr<Join> lookup_; // Selective: the map's keys (LeftOuterSemi probe = "is in the map")
    bool lookup_has_null_ = false;
    void trySwitchFromInitState();
    void trySwitchFromAdjustState(size_t total_rows, size_t hit_rows);
    void trySwitchBackAdjustState(size_t block_rows);
    Block getPassThroughBlock(const Block &block) const;
    void buildLookup();
};

// ---------------------------------------------------------------- packet codec (f1)
// CHBlockChunkCodec / CHBlockChunkCodecV1 (Flash/Coprocessor/CHBlockChunkCodec.cpp:134-258,
// CHBlockChunkCodecV1.cpp:370-583) over tfg_codec_*: the packet is a device buffer.  Const
// columns are materialised first (WriteColumnData).  encode writes NONE packets (LZ4 frames via
// tfg_codec_compress); decode accepts NONE, LZ4 and ZSTD (HIGH_COMPRESSION) packets, decompressed
// on the device.  encode(vector<Block>) writes one part of the concatenated rows (the reference
// writes one part per block; decode accepts both).

class CHBlockChunkCodecV1 {
public:
    CHBlockChunkCodecV1(Context &ctx, Block header) : ctx_(ctx), header_(std::move(header)) {}
    DevicePacket encode(const Block &block); // nothing (empty packet) when the block has no rows
    DevicePacket encode(const std::vector<Block> &blocks);
    static Block decode(Context &ctx, const Block &header, const DevicePacket &packet);
    size_t encoded_rows = 0;
    size_t original_size = 0;

private:
    Context &ctx_;
    Block header_;
};

class CHBlockChunkCodec {
public:
    explicit CHBlockChunkCodec(Context &ctx, Block header = Block()) : ctx_(ctx), header_(std::move(header)) {}
    DevicePacket encode(const Block &block); // CHBlockChunkCodecStream::encode
    Block decode(const DevicePacket &packet) const;

private:
    Context &ctx_;
    Block header_;
};

// shared by both codecs: version = TFG_CODEC_CHBLOCK / TFG_CODEC_V1
DevicePacket encodeBlockPacket(Context &ctx, const Block &block, int version);
Block decodeBlockPacket(Context &ctx, const Block &header, const uint8_t *packet, size_t bytes, int version);

// ---------------------------------------------------------------- streams (IBlockInputStream)
class IBlockInputStream {
public:
    virtual ~IBlockInputStream() = default;
    virtual std::string getName() const = 0;
    virtual Block getHeader() const = 0;
    virtual Block read() = 0; // empty Block = end of stream
    virtual void readPrefix() {}
    virtual void readSuffix() {}
};
using BlockInputStreamPtr = std::shared_ptr<IBlockInputStream>;

class BlocksListBlockInputStream : public IBlockInputStream {
public:
    explicit BlocksListBlockInputStream(std::vector<Block> blocks) : blocks_(std::move(blocks)) {}
    std::string getName() const override { return "BlocksList"; }
    Block getHeader() const override { return blocks_.empty() ? Block() : blocks_[0].cloneEmpty(); }
    Block read() override { return pos_ < blocks_.size() ? blocks_[pos_++] : Block(); }

private:
    std::vector<Block> blocks_;
    size_t pos_ = 0;
};

// FilterBlockInputStream: skips blocks the filter empties (DataStreams/FilterBlockInputStream.cpp)
class FilterBlockInputStream : public IBlockInputStream {
public:
    FilterBlockInputStream(Context &ctx, BlockInputStreamPtr input, ExpressionActionsPtr expression,
                           const std::string &filter_column);
    std::string getName() const override { return "Filter"; }
    Block getHeader() const override { return action_.getHeader(); }
    Block read() override;

private:
    BlockInputStreamPtr input_;
    FilterTransformAction action_;
};

// AggregatingBlockInputStream: consumes the whole input, then returns the result block
// (DataStreams/AggregatingBlockInputStream.cpp).  For the fused filter -> aggregation form
// (no mask materialised) use Aggregator::executeOnBlockFiltered directly.
class AggregatingBlockInputStream : public IBlockInputStream {
public:
    AggregatingBlockInputStream(Context &ctx, BlockInputStreamPtr input, const Aggregator::Params &params,
                                bool final = true);
    std::string getName() const override { return "Aggregating"; }
    Block getHeader() const override;
    Block read() override;

private:
    Context &ctx_;
    BlockInputStreamPtr input_;
    Aggregator aggregator_;
    bool final_;
    bool done_ = false;
    mutable Block header_;
};

// HashJoinProbeBlockInputStream: joinBlock per probe block (DataStreams/HashJoinProbeBlockInputStream.cpp)
class HashJoinProbeBlockInputStream : public IBlockInputStream {
public:
    HashJoinProbeBlockInputStream(BlockInputStreamPtr input, std::shared_ptr<Join> join)
        : input_(std::move(input)), join_(std::move(join)) {}
    std::string getName() const override { return "HashJoinProbe"; }
    Block getHeader() const override { return input_->getHeader(); }
    Block read() override;

private:
    BlockInputStreamPtr input_;
    std::shared_ptr<Join> join_;
};

} // namespace tfa
