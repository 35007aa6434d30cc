// pipeline.h — the pipeline-engine boundary of the hot path: SourceOp / TransformOp / SinkOp
// chained by a PipelineExec, the reference's default execution model
// (Flash/executeQuery.cpp:181-197 picks the pipeline engine; Operators/Operator.h:32-173 the
// operator contract; Flash/Pipeline/Exec/PipelineExec.cpp:120-180 the fetch / transform / write
// loop).  The operators on the path keep the reference's names, status contract and block flow:
//
//   FilterTransformOp              Operators/FilterTransformOp.cpp:20-38
//   ExpressionTransformOp          Operators/ExpressionTransformOp.cpp
//   AggregateBuildSinkOp           Operators/AggregateBuildSinkOp.cpp:20-52
//   AggregateConvergentSourceOp    Operators/AggregateConvergentSourceOp.cpp:20-38
//   AggregateContext               Operators/AggregateContext.cpp:80-215
//   HashJoinBuildSink              Operators/HashJoinBuildSink.cpp:20-56
//   HashJoinProbeTransformOp       Operators/HashJoinProbeTransformOp.cpp:70-235
//   ExchangeSenderSinkOp           Operators/ExchangeSenderSinkOp.cpp:20-85
//   ExchangeReceiverSourceOp       Operators/ExchangeReceiverSourceOp.cpp:63-110
//   GetResultSinkOp                Operators/GetResultSinkOp.h
//
// MI355X-first differences: every operator's work is device work on the Context's HIP stream,
// so one host thread drives all PipelineExecs of a pipeline round-robin (runPipelineExecs — the
// TaskScheduler's role); the build tasks of an AggregateContext / Join share ONE device table
// (the GPU is the parallel engine, so there are no per-thread maps to merge); no spill states
// (IO_IN / IO_OUT are honoured by the executor but the operators here never return them:
// HBM holds the tables).
#pragma once
#include <atomic>
#include <deque>
#include <mutex>

#include "tfa_host.h"

namespace tfa {

enum class OperatorStatus {
    FINISHED,        // finish status (sinks only)
    CANCELLED,       // cancel status
    WAITING,         // waiting status: poll await()
    WAIT_FOR_NOTIFY, // waiting status: parked until notify()
    IO_IN,           // io status: executeIO()
    IO_OUT,
    NEED_INPUT,      // running: TransformOp / SinkOp needs a block
    HAS_OUTPUT,      // running: SourceOp / TransformOp produced a block
};
const char *toString(OperatorStatus s);

class PipelineExecutorContext {
public:
    void cancel() { cancelled_ = true; }
    bool isCancelled() const { return cancelled_; }

private:
    std::atomic<bool> cancelled_{false};
};

struct OperatorProfileInfo {
    uint64_t blocks = 0;
    uint64_t rows = 0;
    uint64_t execution_ns = 0; // host time inside the operator (device work is asynchronous)
};

class Operator {
public:
    Operator(PipelineExecutorContext &exec_context, Context &ctx) : exec_context(exec_context), ctx_(ctx) {}
    virtual ~Operator() = default;
    OperatorStatus executeIO(); // NEED_INPUT / HAS_OUTPUT / FINISHED
    OperatorStatus await();     // NEED_INPUT / HAS_OUTPUT / FINISHED / WAITING
    void notify();
    void operatePrefix();
    void operateSuffix();
    virtual std::string getName() const = 0;
    Block getHeader() const { return header; }
    void setHeader(const Block &h) { header = h; }
    const OperatorProfileInfo &getProfileInfo() const { return profile_info; }
    // true when the operator accepts a block whose info.selective is set (BlockInfo.h:47-49)
    virtual bool canHandleSelectiveBlock() const { return false; }

protected:
    virtual void operatePrefixImpl() {}
    virtual void operateSuffixImpl() {}
    virtual OperatorStatus executeIOImpl();
    virtual OperatorStatus awaitImpl();
    virtual void notifyImpl() {}
    void account(const Block *block, uint64_t t0_ns);

    PipelineExecutorContext &exec_context;
    Context &ctx_;
    Block header;
    OperatorProfileInfo profile_info;
};

// The running status of a source is HAS_OUTPUT: a block, or (once exhausted) an empty Block,
// which flows down the pipeline as the end-of-input marker.
class SourceOp : public Operator {
public:
    using Operator::Operator;
    OperatorStatus read(Block &block);

protected:
    virtual OperatorStatus readImpl(Block &block) = 0;
};

class TransformOp : public Operator {
public:
    using Operator::Operator;
    // HAS_OUTPUT (block filled) or NEED_INPUT: output the operator holds without new input
    OperatorStatus tryOutput(Block &block);
    // in place; HAS_OUTPUT passes the block on (an empty Block too), NEED_INPUT asks for more
    OperatorStatus transform(Block &block);
    void transformHeader(Block &h) {
        transformHeaderImpl(h);
        setHeader(h);
    }

protected:
    virtual OperatorStatus tryOutputImpl(Block &) { return OperatorStatus::NEED_INPUT; }
    virtual OperatorStatus transformImpl(Block &block) = 0;
    virtual void transformHeaderImpl(Block &h) = 0;
};

// The running status of a sink is NEED_INPUT; FINISHED once the end-of-input block is written.
class SinkOp : public Operator {
public:
    using Operator::Operator;
    OperatorStatus prepare();
    OperatorStatus write(Block &&block);

protected:
    virtual OperatorStatus prepareImpl() { return OperatorStatus::NEED_INPUT; }
    virtual OperatorStatus writeImpl(Block &&block) = 0;
};

using SourceOpPtr = std::unique_ptr<SourceOp>;
using TransformOpPtr = std::unique_ptr<TransformOp>;
using TransformOps = std::vector<TransformOpPtr>;
using SinkOpPtr = std::unique_ptr<SinkOp>;

//   sink.prepare -> transform.tryOutput (last to first) -> source.read -> transforms -> sink.write
class PipelineExec {
public:
    PipelineExec(SourceOpPtr source, TransformOps transforms, SinkOpPtr sink);
    void executePrefix();
    void executeSuffix();
    OperatorStatus execute();   // FINISHED / NEED_INPUT / CANCELLED / a waiting or io status
    OperatorStatus executeIO(); // after IO_IN / IO_OUT
    OperatorStatus await();     // after WAITING
    void notify();              // after WAIT_FOR_NOTIFY
    const SourceOp &source() const { return *source_op_; }
    const SinkOp &sink() const { return *sink_op_; }
    const TransformOps &transforms() const { return transform_ops_; }

private:
    SourceOpPtr source_op_;
    TransformOps transform_ops_;
    SinkOpPtr sink_op_;
    Operator *io_op_ = nullptr;
    Operator *awaitable_ = nullptr;
    Operator *waiting_for_notify_ = nullptr;
    OperatorStatus fetchBlock(Block &block, size_t &start_transform);
    OperatorStatus handle(Operator *op, OperatorStatus s, OperatorStatus expect, bool last);
};
using PipelineExecPtr = std::unique_ptr<PipelineExec>;

// Drives every PipelineExec of one pipeline (one per degree of concurrency) round-robin on this
// thread until each returns FINISHED: IO statuses run executeIO, WAITING polls await, and a
// WAIT_FOR_NOTIFY exec is parked until its op is notified (here: retried once every other exec
// has made a step).  Throws on CANCELLED (exec_context.cancel()) or when no exec can progress.
void runPipelineExecs(PipelineExecutorContext &exec_context, std::vector<PipelineExecPtr> &execs);

// ---------------------------------------------------------------- sources / sinks
// A list of blocks (BlockInputStreamSourceOp over a BlocksListBlockInputStream; the mock table
// scan of the reference's operator tests).
class BlocksSourceOp : public SourceOp {
public:
    BlocksSourceOp(PipelineExecutorContext &exec, Context &ctx, Block header, std::vector<Block> blocks);
    std::string getName() const override { return "BlocksSourceOp"; }

protected:
    OperatorStatus readImpl(Block &block) override;

private:
    std::vector<Block> blocks_;
    size_t pos_ = 0;
};

// BlockInputStreamSourceOp (Operators/BlockInputStreamSourceOp.cpp): an IBlockInputStream as a source
class BlockInputStreamSourceOp : public SourceOp {
public:
    BlockInputStreamSourceOp(PipelineExecutorContext &exec, Context &ctx, BlockInputStreamPtr stream);
    std::string getName() const override { return "BlockInputStreamSourceOp"; }

protected:
    OperatorStatus readImpl(Block &block) override;
    void operatePrefixImpl() override { stream_->readPrefix(); }
    void operateSuffixImpl() override { stream_->readSuffix(); }

private:
    BlockInputStreamPtr stream_;
};

// GetResultSinkOp: hands every block to a result handler (the query's result queue).
class GetResultSinkOp : public SinkOp {
public:
    using ResultHandler = std::function<void(const Block &)>;
    GetResultSinkOp(PipelineExecutorContext &exec, Context &ctx, ResultHandler handler);
    std::string getName() const override { return "GetResultSinkOp"; }

protected:
    OperatorStatus writeImpl(Block &&block) override;

private:
    ResultHandler handler_;
};

// ---------------------------------------------------------------- transforms (a4, a5)
class FilterTransformOp : public TransformOp {
public:
    FilterTransformOp(PipelineExecutorContext &exec, Context &ctx, const Block &input_header,
                      ExpressionActionsPtr expression, const std::string &filter_column);
    std::string getName() const override { return "FilterTransformOp"; }

protected:
    OperatorStatus transformImpl(Block &block) override;
    void transformHeaderImpl(Block &h) override { h = action_.getHeader(); }

private:
    FilterTransformAction action_;
    FilterPtr filter_ignored_;
};

class ExpressionTransformOp : public TransformOp {
public:
    ExpressionTransformOp(PipelineExecutorContext &exec, Context &ctx, ExpressionActionsPtr expression);
    std::string getName() const override { return "ExpressionTransformOp"; }

protected:
    OperatorStatus transformImpl(Block &block) override;
    void transformHeaderImpl(Block &h) override;

private:
    ExpressionActionsPtr expression_;
};

// ---------------------------------------------------------------- aggregation (a9-a17)
// AggregateContext: the build side's shared state.  Every build task (index) folds into one
// device Aggregator (buildOnBlock serialises on a mutex: the device table is the parallel part);
// initConvergent converts it once to the result block, which readForConvergent hands out as
// `concurrency` row ranges (one per convergent source), then empty Blocks.
class AggregateContext {
public:
    AggregateContext(Context &ctx, const Aggregator::Params &params, size_t concurrency, bool final = true);
    void buildOnBlock(size_t index, const Block &block);
    // fused FilterTransformAction -> Aggregator for one `column Op constant` predicate
    void buildOnBlockFiltered(size_t index, const Block &block, const std::string &pred, int op, Field constant);
    void initConvergent();
    Block readForConvergent(size_t index);
    Block getHeader() const { return header_; }
    size_t getTotalBuildRows(size_t index) const { return index < build_rows_.size() ? build_rows_[index] : 0; }
    size_t concurrency() const { return concurrency_; }
    bool isConvergentReady() const { return converged_; }
    void finishBuild(size_t index); // one build task is done
    bool allBuildFinished() const { return finished_builds_ == concurrency_; }

private:
    Context &ctx_;
    Aggregator agg_;
    size_t concurrency_;
    bool final_;
    Block header_;
    std::mutex mu_;
    std::vector<size_t> build_rows_;
    size_t finished_builds_ = 0;
    bool converged_ = false;
    std::vector<Block> slices_;
    std::vector<bool> read_;
};
using AggregateContextPtr = std::shared_ptr<AggregateContext>;

class AggregateBuildSinkOp : public SinkOp {
public:
    AggregateBuildSinkOp(PipelineExecutorContext &exec, Context &ctx, AggregateContextPtr agg_context, size_t index);
    // pushes a `pred Op constant` filter into the build (the fused filter -> GROUP BY kernels)
    void setPushedDownFilter(const std::string &pred, int op, Field constant);
    std::string getName() const override { return "AggregateBuildSinkOp"; }

protected:
    OperatorStatus writeImpl(Block &&block) override;

private:
    AggregateContextPtr agg_context_;
    size_t index_;
    bool has_filter_ = false;
    std::string pred_;
    int op_ = 0;
    Field constant_;
};

class AggregateConvergentSourceOp : public SourceOp {
public:
    AggregateConvergentSourceOp(PipelineExecutorContext &exec, Context &ctx, AggregateContextPtr agg_context,
                                size_t index);
    std::string getName() const override { return "AggregateConvergentSourceOp"; }
    uint64_t totalRows() const { return total_rows_; }

protected:
    OperatorStatus readImpl(Block &block) override;

private:
    AggregateContextPtr agg_context_;
    size_t index_;
    uint64_t total_rows_ = 0;
};

// ---------------------------------------------------------------- hash join (a18-a21)
// JoinBuildContext: the Join and the number of build tasks still running (Join::finishOneBuild
// of the reference returns true for the last one, which finalizes the table).
class JoinBuildContext {
public:
    JoinBuildContext(Context &ctx, std::shared_ptr<Join> join, size_t build_concurrency, Block build_header);
    void insertFromBlock(const Block &block);
    bool finishOneBuild(); // true for the last build task (the table is then finalized)
    bool isFinalized() const { return finalized_; }
    const std::shared_ptr<Join> &join() const { return join_; }

private:
    Context &ctx_;
    std::shared_ptr<Join> join_;
    size_t active_;
    Block build_header_;
    bool finalized_ = false;
    bool inserted_ = false;
    std::mutex mu_;
};
using JoinBuildContextPtr = std::shared_ptr<JoinBuildContext>;

class HashJoinBuildSink : public SinkOp {
public:
    HashJoinBuildSink(PipelineExecutorContext &exec, Context &ctx, JoinBuildContextPtr join, size_t op_index);
    std::string getName() const override { return "HashJoinBuildSink"; }

protected:
    OperatorStatus writeImpl(Block &&block) override;

private:
    JoinBuildContextPtr join_;
    size_t op_index_;
};

// Probe blocks joined against the finalized table; output larger than max_block_size rows is
// handed out in max_block_size slices through tryOutput (ProbeProcessInfo's block splitting).
class HashJoinProbeTransformOp : public TransformOp {
public:
    HashJoinProbeTransformOp(PipelineExecutorContext &exec, Context &ctx, JoinBuildContextPtr join, size_t op_index,
                             size_t max_block_size);
    std::string getName() const override { return "HashJoinProbeTransformOp"; }
    uint64_t joinedRows() const { return joined_rows_; }

protected:
    OperatorStatus transformImpl(Block &block) override;
    OperatorStatus tryOutputImpl(Block &block) override;
    void transformHeaderImpl(Block &h) override;

private:
    JoinBuildContextPtr join_;
    size_t op_index_;
    size_t max_block_size_;
    std::deque<Block> pending_;
    bool finished_ = false;
    uint64_t joined_rows_ = 0;
};

// ---------------------------------------------------------------- exchange (a22-a24, e)
// ExchangeReceiver: the blocks that arrived for this node (one queue; the receiver sources of a
// pipeline pop from it).  finish() marks the end of every sender's stream.
class ExchangeReceiver {
public:
    // stream: the fine-grained shuffle stream id of the chunk the block came in (0 otherwise);
    // the reference routes such chunks to per-stream channels (ExchangeReceiver.cpp, fine-grained
    // msg channels), read by the stream's own source
    void push(Block block, uint32_t stream = 0);
    void finish();
    bool tryPop(Block &block); // false when nothing is queued
    // the first queued block of a stream s with s % stride == index (fine-grained sources)
    bool tryPop(Block &block, uint32_t stride, uint32_t index);
    bool finished() const { return finished_; }

private:
    std::mutex mu_;
    std::deque<std::pair<uint32_t, Block>> queue_;
    std::atomic<bool> finished_{false};
};
using ExchangeReceiverPtr = std::shared_ptr<ExchangeReceiver>;

// The tunnels of an ExchangeSender: per-partition blocks from every sender task of this node
// are collected; when the last sender finishes, the partitions go out — through an MPPExchange
// (RCCL all-to-all; partition p to rank p) into `receiver`, or, without one, partition
// `local_partition` straight into `receiver` and the others to `remote` (the tunnels to other
// nodes, e.g. a test's capture) with their fine-grained stream ids, so the remote receiver routes
// each block to the stream that aggregates its keys (MPPTunnelSetWriter.cpp:365-400 carries the
// stream id in the packet's chunks).
class MPPTunnelSet {
public:
    using RemoteSink = std::function<void(uint32_t part, Block &&, uint32_t stream)>;
    MPPTunnelSet(Context &ctx, uint32_t partition_num, size_t sender_concurrency, ExchangeReceiverPtr receiver,
                 MPPExchange *exchange = nullptr, uint32_t local_partition = 0, RemoteSink remote = nullptr);
    void write(uint32_t part, Block &&block, uint32_t stream = 0); // stream: fine-grained stream id
    void finishOneSender(); // the last one sends
    uint32_t partitionNum() const { return partition_num_; }

private:
    Context &ctx_;
    uint32_t partition_num_;
    size_t active_;
    ExchangeReceiverPtr receiver_;
    MPPExchange *exchange_;
    uint32_t local_partition_;
    RemoteSink remote_;
    std::vector<std::vector<Block>> parts_;
    std::vector<std::vector<uint32_t>> streams_; // the stream id of each block of parts_
    std::mutex mu_;
};
using MPPTunnelSetPtr = std::shared_ptr<MPPTunnelSet>;

// ExchangeSenderSinkOp with a HashPartitionWriter (HashPartitionWriter.cpp:76-204): rows are
// buffered to batch_send_min_limit, weak-hashed on the partition keys, scattered, and written
// to the tunnels; the end-of-input block flushes.
class ExchangeSenderSinkOp : public SinkOp {
public:
    // fine_grained_stream_count > 0: a FineGrainedShuffleWriter (newMPPExchangeWriter.cpp:66-78)
    // with batches of fine_grained_batch_size rows per stream
    ExchangeSenderSinkOp(PipelineExecutorContext &exec, Context &ctx, MPPTunnelSetPtr tunnels,
                         std::vector<size_t> partition_col_ids, std::vector<int> collators = {},
                         int64_t batch_send_min_limit = -1, uint32_t fine_grained_stream_count = 0,
                         uint64_t fine_grained_batch_size = 8192);
    std::string getName() const override { return "ExchangeSenderSinkOp"; }
    uint64_t totalRows() const { return total_rows_; }

protected:
    OperatorStatus writeImpl(Block &&block) override;
    void operatePrefixImpl() override;

private:
    MPPTunnelSetPtr tunnels_;
    std::unique_ptr<HashPartitionWriter> writer_;
    std::unique_ptr<FineGrainedShuffleWriter> fg_writer_;
    std::shared_ptr<Block> fg_header_; // the chunks' schema (the first block's), shared with the sink
    std::vector<size_t> partition_col_ids_;
    std::vector<int> collators_;
    int64_t limit_;
    uint32_t fg_streams_;
    uint64_t fg_batch_;
    uint64_t total_rows_ = 0;
};

class ExchangeReceiverSourceOp : public SourceOp {
public:
    // stride > 0: reads only the fine-grained streams s with s % stride == index
    ExchangeReceiverSourceOp(PipelineExecutorContext &exec, Context &ctx, ExchangeReceiverPtr receiver, Block header,
                             uint32_t stride = 0, uint32_t index = 0);
    std::string getName() const override { return "ExchangeReceiverSourceOp"; }

protected:
    OperatorStatus readImpl(Block &block) override;
    OperatorStatus awaitImpl() override;

private:
    ExchangeReceiverPtr receiver_;
    uint32_t stride_, index_;
    Block next_;
    bool has_next_ = false;
};

// A zero-row block of the header's columns with allocated (1-byte) buffers, as device code expects.
Block emptyLike(Context &ctx, const Block &header);

// Rows [offset, offset + rows) of a block (device gather; String / Nullable columns included).
Block sliceBlock(Context &ctx, const Block &block, size_t offset, size_t rows);

} // namespace tfa
