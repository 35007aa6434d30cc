// pipeline.cpp — SourceOp / TransformOp / SinkOp, PipelineExec and the hot-path operators
// (see pipeline.h for the reference map).
#include "pipeline.h"

#include <chrono>
#include <thread>

namespace tfa {

namespace {
uint64_t now_ns() {
    return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
               std::chrono::steady_clock::now().time_since_epoch())
        .count();
}

void expectStatus(const Operator &op, const char *method, OperatorStatus s, std::initializer_list<OperatorStatus> ok) {
    // running statuses are checked; cancel / waiting / io statuses may come from any method
    if (s == OperatorStatus::CANCELLED || s == OperatorStatus::WAITING || s == OperatorStatus::WAIT_FOR_NOTIFY ||
        s == OperatorStatus::IO_IN || s == OperatorStatus::IO_OUT)
        return;
    for (OperatorStatus o : ok)
        if (o == s) return;
    throw Exception(op.getName() + "::" + method + " returned " + toString(s), ErrorCodes::LOGICAL_ERROR);
}

void checkStructure(const Operator &op, const Block &block) {
    const Block h = op.getHeader();
    if (!h || !block) return;
    bool same = h.columns() == block.columns();
    for (size_t i = 0; same && i < h.columns(); ++i)
        same = h.safeGetByPosition(i).name == block.safeGetByPosition(i).name &&
               h.safeGetByPosition(i).type.type == block.safeGetByPosition(i).type.type;
    if (!same)
        throw Exception(op.getName() + " output does not match its header", ErrorCodes::LOGICAL_ERROR);
}

} // namespace

// a zero-row block of the header's columns with allocated (1-byte) buffers, as device code expects
Block emptyLike(Context &ctx, const Block &header) {
    Block out;
    for (const auto &c : header.getColumnsWithTypeAndName()) {
        auto z = std::make_shared<IColumn>();
        z->type = c.type;
        z->data = std::make_shared<DeviceBuffer>(ctx, 1);
        if (c.type.isString()) {
            z->offsets = std::make_shared<DeviceBuffer>(ctx, 8);
        }
        if (c.type.nullable) z->nullmap = std::make_shared<DeviceBuffer>(ctx, 1);
        out.insert({z, z->type, c.name});
    }
    return out;
}

const char *toString(OperatorStatus s) {
    switch (s) {
    case OperatorStatus::FINISHED: return "FINISHED";
    case OperatorStatus::CANCELLED: return "CANCELLED";
    case OperatorStatus::WAITING: return "WAITING";
    case OperatorStatus::WAIT_FOR_NOTIFY: return "WAIT_FOR_NOTIFY";
    case OperatorStatus::IO_IN: return "IO_IN";
    case OperatorStatus::IO_OUT: return "IO_OUT";
    case OperatorStatus::NEED_INPUT: return "NEED_INPUT";
    case OperatorStatus::HAS_OUTPUT: return "HAS_OUTPUT";
    }
    return "?";
}

// ================================================================ Operator (Operators/Operator.cpp)
void Operator::account(const Block *block, uint64_t t0) {
    profile_info.execution_ns += now_ns() - t0;
    if (block && *block) {
        ++profile_info.blocks;
        profile_info.rows += block->rows();
    }
}

OperatorStatus Operator::executeIOImpl() {
    throw Exception(getName() + " has no IO stage", ErrorCodes::NOT_IMPLEMENTED);
}
OperatorStatus Operator::awaitImpl() { throw Exception(getName() + " cannot await", ErrorCodes::NOT_IMPLEMENTED); }

void Operator::operatePrefix() {
    const uint64_t t0 = now_ns();
    operatePrefixImpl();
    account(nullptr, t0);
}

void Operator::operateSuffix() {
    const uint64_t t0 = now_ns();
    operateSuffixImpl();
    account(nullptr, t0);
}

OperatorStatus Operator::executeIO() {
    if (exec_context.isCancelled()) return OperatorStatus::CANCELLED;
    const uint64_t t0 = now_ns();
    const OperatorStatus s = executeIOImpl();
    expectStatus(*this, "executeIO", s, {OperatorStatus::FINISHED, OperatorStatus::NEED_INPUT, OperatorStatus::HAS_OUTPUT});
    account(nullptr, t0);
    return s;
}

OperatorStatus Operator::await() {
    const OperatorStatus s = awaitImpl();
    expectStatus(*this, "await", s, {OperatorStatus::FINISHED, OperatorStatus::NEED_INPUT, OperatorStatus::HAS_OUTPUT});
    return s;
}

void Operator::notify() { notifyImpl(); }

OperatorStatus SourceOp::read(Block &block) {
    if (exec_context.isCancelled()) return OperatorStatus::CANCELLED;
    const uint64_t t0 = now_ns();
    const OperatorStatus s = readImpl(block);
    expectStatus(*this, "read", s, {OperatorStatus::HAS_OUTPUT});
    if (s == OperatorStatus::HAS_OUTPUT) checkStructure(*this, block);
    account(s == OperatorStatus::HAS_OUTPUT ? &block : nullptr, t0);
    return s;
}

OperatorStatus TransformOp::transform(Block &block) {
    if (exec_context.isCancelled()) return OperatorStatus::CANCELLED;
    if (block && block.info.selective && !canHandleSelectiveBlock())
        throw Exception(getName() + " cannot handle selective block", ErrorCodes::LOGICAL_ERROR);
    const uint64_t t0 = now_ns();
    const OperatorStatus s = transformImpl(block);
    expectStatus(*this, "transform", s, {OperatorStatus::NEED_INPUT, OperatorStatus::HAS_OUTPUT});
    if (s == OperatorStatus::HAS_OUTPUT) checkStructure(*this, block);
    account(s == OperatorStatus::HAS_OUTPUT ? &block : nullptr, t0);
    return s;
}

OperatorStatus TransformOp::tryOutput(Block &block) {
    if (exec_context.isCancelled()) return OperatorStatus::CANCELLED;
    const uint64_t t0 = now_ns();
    const OperatorStatus s = tryOutputImpl(block);
    expectStatus(*this, "tryOutput", s, {OperatorStatus::NEED_INPUT, OperatorStatus::HAS_OUTPUT});
    if (s == OperatorStatus::HAS_OUTPUT) checkStructure(*this, block);
    account(s == OperatorStatus::HAS_OUTPUT ? &block : nullptr, t0);
    return s;
}

OperatorStatus SinkOp::prepare() {
    if (exec_context.isCancelled()) return OperatorStatus::CANCELLED;
    const uint64_t t0 = now_ns();
    const OperatorStatus s = prepareImpl();
    expectStatus(*this, "prepare", s, {OperatorStatus::NEED_INPUT, OperatorStatus::FINISHED});
    account(nullptr, t0);
    return s;
}

OperatorStatus SinkOp::write(Block &&block) {
    if (exec_context.isCancelled()) return OperatorStatus::CANCELLED;
    if (block && block.info.selective && !canHandleSelectiveBlock())
        throw Exception(getName() + " cannot handle selective block", ErrorCodes::LOGICAL_ERROR);
    const uint64_t t0 = now_ns();
    const Block *seen = block ? &block : nullptr;
    const size_t rows = seen ? block.rows() : 0;
    const OperatorStatus s = writeImpl(std::move(block));
    expectStatus(*this, "write", s, {OperatorStatus::NEED_INPUT, OperatorStatus::FINISHED});
    profile_info.execution_ns += now_ns() - t0;
    if (seen) {
        ++profile_info.blocks;
        profile_info.rows += rows;
    }
    return s;
}

// ================================================================ PipelineExec (PipelineExec.cpp)
PipelineExec::PipelineExec(SourceOpPtr source, TransformOps transforms, SinkOpPtr sink)
    : source_op_(std::move(source)), transform_ops_(std::move(transforms)), sink_op_(std::move(sink)) {
    if (!source_op_ || !sink_op_) throw Exception("a pipeline needs a source and a sink", ErrorCodes::BAD_ARGUMENTS);
}

void PipelineExec::executePrefix() {
    sink_op_->operatePrefix();
    for (auto it = transform_ops_.rbegin(); it != transform_ops_.rend(); ++it) (*it)->operatePrefix();
    source_op_->operatePrefix();
}

void PipelineExec::executeSuffix() {
    sink_op_->operateSuffix();
    for (auto it = transform_ops_.rbegin(); it != transform_ops_.rend(); ++it) (*it)->operateSuffix();
    source_op_->operateSuffix();
}

// HANDLE_OP_STATUS / HANDLE_LAST_OP_STATUS: `expect` continues the caller (returned as is);
// io and waiting statuses record the operator to resume; anything else returns
OperatorStatus PipelineExec::handle(Operator *op, OperatorStatus s, OperatorStatus expect, bool last) {
    switch (s) {
    case OperatorStatus::IO_IN:
    case OperatorStatus::IO_OUT: io_op_ = op; return s;
    case OperatorStatus::WAITING: awaitable_ = op; return s;
    case OperatorStatus::WAIT_FOR_NOTIFY: waiting_for_notify_ = op; return s;
    default: return last ? s : s == expect ? expect : s;
    }
}

OperatorStatus PipelineExec::fetchBlock(Block &block, size_t &start_transform) {
    OperatorStatus s = handle(sink_op_.get(), sink_op_->prepare(), OperatorStatus::NEED_INPUT, false);
    if (s != OperatorStatus::NEED_INPUT) return s;
    for (int64_t i = (int64_t)transform_ops_.size() - 1; i >= 0; --i) {
        s = handle(transform_ops_[i].get(), transform_ops_[i]->tryOutput(block), OperatorStatus::NEED_INPUT, false);
        start_transform = (size_t)i + 1; // a block from op i continues at op i + 1
        if (s != OperatorStatus::NEED_INPUT) return s;
    }
    start_transform = 0;
    return handle(source_op_.get(), source_op_->read(block), OperatorStatus::HAS_OUTPUT, true);
}

OperatorStatus PipelineExec::execute() {
    if (io_op_ || awaitable_ || waiting_for_notify_)
        throw Exception("execute() while an operator awaits io / a wait / a notify", ErrorCodes::LOGICAL_ERROR);
    Block block;
    size_t start = 0;
    OperatorStatus s = fetchBlock(block, start);
    if (s != OperatorStatus::HAS_OUTPUT) return s;
    if (block && block.rows() == 0) return OperatorStatus::NEED_INPUT;
    for (size_t i = start; i < transform_ops_.size(); ++i) {
        s = handle(transform_ops_[i].get(), transform_ops_[i]->transform(block), OperatorStatus::HAS_OUTPUT, false);
        if (s != OperatorStatus::HAS_OUTPUT) return s;
        if (block && block.rows() == 0) return OperatorStatus::NEED_INPUT;
    }
    return handle(sink_op_.get(), sink_op_->write(std::move(block)), OperatorStatus::NEED_INPUT, true);
}

OperatorStatus PipelineExec::executeIO() {
    if (!io_op_) throw Exception("executeIO() without an io operator", ErrorCodes::LOGICAL_ERROR);
    Operator *op = io_op_;
    const OperatorStatus s = op->executeIO();
    if (s == OperatorStatus::IO_IN || s == OperatorStatus::IO_OUT) return s;
    io_op_ = nullptr;
    if (s == OperatorStatus::WAITING) awaitable_ = op;
    if (s == OperatorStatus::WAIT_FOR_NOTIFY) waiting_for_notify_ = op;
    return s;
}

OperatorStatus PipelineExec::await() {
    if (!awaitable_) throw Exception("await() without a waiting operator", ErrorCodes::LOGICAL_ERROR);
    Operator *op = awaitable_;
    const OperatorStatus s = op->await();
    if (s == OperatorStatus::WAITING) return s;
    awaitable_ = nullptr;
    if (s == OperatorStatus::IO_IN || s == OperatorStatus::IO_OUT) io_op_ = op;
    if (s == OperatorStatus::WAIT_FOR_NOTIFY) waiting_for_notify_ = op;
    return s;
}

void PipelineExec::notify() {
    if (!waiting_for_notify_) throw Exception("notify() without a parked operator", ErrorCodes::LOGICAL_ERROR);
    waiting_for_notify_->notify();
    waiting_for_notify_ = nullptr;
}

void runPipelineExecs(PipelineExecutorContext &exec_context, std::vector<PipelineExecPtr> &execs) {
    for (auto &e : execs) e->executePrefix();
    std::vector<OperatorStatus> last(execs.size(), OperatorStatus::NEED_INPUT);
    std::vector<bool> done(execs.size(), false);
    size_t remaining = execs.size();
    auto stalled_since = std::chrono::steady_clock::now();
    while (remaining) {
        bool progress = false;
        for (size_t i = 0; i < execs.size(); ++i) {
            if (done[i]) continue;
            PipelineExec &e = *execs[i];
            OperatorStatus s;
            switch (last[i]) {
            case OperatorStatus::IO_IN:
            case OperatorStatus::IO_OUT: s = e.executeIO(); break;
            case OperatorStatus::WAITING: s = e.await(); break;
            case OperatorStatus::WAIT_FOR_NOTIFY: e.notify(); s = e.execute(); break;
            default: s = e.execute(); break;
            }
            if (s == OperatorStatus::CANCELLED || exec_context.isCancelled())
                throw Exception("pipeline cancelled", ErrorCodes::LOGICAL_ERROR);
            if (s == OperatorStatus::FINISHED) {
                done[i] = true;
                --remaining;
            }
            if (s != OperatorStatus::WAITING && s != OperatorStatus::WAIT_FOR_NOTIFY) progress = true;
            last[i] = s;
        }
        if (progress) {
            stalled_since = std::chrono::steady_clock::now();
        } else {
            if (std::chrono::steady_clock::now() - stalled_since > std::chrono::seconds(60))
                throw Exception("pipeline stalled: every exec is waiting", ErrorCodes::LOGICAL_ERROR);
            std::this_thread::yield();
        }
    }
    for (auto &e : execs) e->executeSuffix();
}

// ================================================================ sources / sinks
BlocksSourceOp::BlocksSourceOp(PipelineExecutorContext &exec, Context &ctx, Block header, std::vector<Block> blocks)
    : SourceOp(exec, ctx), blocks_(std::move(blocks)) {
    setHeader(header.cloneEmpty());
}

OperatorStatus BlocksSourceOp::readImpl(Block &block) {
    block = pos_ < blocks_.size() ? blocks_[pos_++] : Block();
    return OperatorStatus::HAS_OUTPUT;
}

BlockInputStreamSourceOp::BlockInputStreamSourceOp(PipelineExecutorContext &exec, Context &ctx,
                                                   BlockInputStreamPtr stream)
    : SourceOp(exec, ctx), stream_(std::move(stream)) {
    setHeader(stream_->getHeader());
}

OperatorStatus BlockInputStreamSourceOp::readImpl(Block &block) {
    block = stream_->read();
    return OperatorStatus::HAS_OUTPUT;
}

GetResultSinkOp::GetResultSinkOp(PipelineExecutorContext &exec, Context &ctx, ResultHandler handler)
    : SinkOp(exec, ctx), handler_(std::move(handler)) {
    if (!handler_) throw Exception("GetResultSinkOp needs a result handler", ErrorCodes::BAD_ARGUMENTS);
}

OperatorStatus GetResultSinkOp::writeImpl(Block &&block) {
    if (!block) return OperatorStatus::FINISHED;
    handler_(block);
    return OperatorStatus::NEED_INPUT;
}

// ================================================================ transforms
FilterTransformOp::FilterTransformOp(PipelineExecutorContext &exec, Context &ctx, const Block &input_header,
                                     ExpressionActionsPtr expression, const std::string &filter_column)
    : TransformOp(exec, ctx), action_(ctx, input_header, std::move(expression), filter_column) {
    Block h = input_header;
    transformHeader(h);
}

// FilterTransformOp::transformImpl: a block the filter empties asks for more input
OperatorStatus FilterTransformOp::transformImpl(Block &block) {
    if (block) return action_.transform(block, filter_ignored_, false) ? OperatorStatus::HAS_OUTPUT : OperatorStatus::NEED_INPUT;
    return OperatorStatus::HAS_OUTPUT;
}

ExpressionTransformOp::ExpressionTransformOp(PipelineExecutorContext &exec, Context &ctx,
                                             ExpressionActionsPtr expression)
    : TransformOp(exec, ctx), expression_(std::move(expression)) {}

void ExpressionTransformOp::transformHeaderImpl(Block &h) {
    Block z = emptyLike(ctx_, h);
    expression_->execute(z);
    h = z.cloneEmpty();
}

OperatorStatus ExpressionTransformOp::transformImpl(Block &block) {
    if (block) expression_->execute(block);
    return OperatorStatus::HAS_OUTPUT;
}

// ================================================================ aggregation
AggregateContext::AggregateContext(Context &ctx, const Aggregator::Params &params, size_t concurrency, bool final)
    : ctx_(ctx), agg_(ctx, params), concurrency_(std::max<size_t>(concurrency, 1)), final_(final),
      build_rows_(std::max<size_t>(concurrency, 1), 0), read_(std::max<size_t>(concurrency, 1), false) {
    header_ = agg_.convertToBlock(final_).cloneEmpty();
}

void AggregateContext::buildOnBlock(size_t index, const Block &block) {
    if (index >= concurrency_) throw Exception("build index out of range", ErrorCodes::BAD_ARGUMENTS);
    std::lock_guard<std::mutex> g(mu_);
    if (converged_) throw Exception("buildOnBlock after initConvergent", ErrorCodes::LOGICAL_ERROR);
    agg_.executeOnBlock(block);
    build_rows_[index] += block.rows();
}

void AggregateContext::buildOnBlockFiltered(size_t index, const Block &block, const std::string &pred, int op,
                                            Field constant) {
    if (index >= concurrency_) throw Exception("build index out of range", ErrorCodes::BAD_ARGUMENTS);
    std::lock_guard<std::mutex> g(mu_);
    if (converged_) throw Exception("buildOnBlock after initConvergent", ErrorCodes::LOGICAL_ERROR);
    agg_.executeOnBlockFiltered(block, pred, op, constant);
    build_rows_[index] += block.rows();
}

void AggregateContext::finishBuild(size_t index) {
    std::lock_guard<std::mutex> g(mu_);
    ++finished_builds_;
}

// the converted result, cut into `concurrency` row ranges (one per convergent source)
void AggregateContext::initConvergent() {
    std::lock_guard<std::mutex> g(mu_);
    if (converged_) return;
    Block all = agg_.convertToBlock(final_);
    const size_t n = all ? all.rows() : 0;
    slices_.clear();
    for (size_t i = 0; i < concurrency_; ++i) {
        const size_t lo = n * i / concurrency_, hi = n * (i + 1) / concurrency_;
        if (concurrency_ == 1) slices_.push_back(all);
        else slices_.push_back(hi > lo ? sliceBlock(ctx_, all, lo, hi - lo) : Block());
    }
    converged_ = true;
}

Block AggregateContext::readForConvergent(size_t index) {
    if (index >= concurrency_) throw Exception("convergent index out of range", ErrorCodes::BAD_ARGUMENTS);
    if (!converged_) initConvergent();
    std::lock_guard<std::mutex> g(mu_);
    if (read_[index]) return Block();
    read_[index] = true;
    Block b = std::move(slices_[index]);
    return b && b.rows() ? b : Block();
}

AggregateBuildSinkOp::AggregateBuildSinkOp(PipelineExecutorContext &exec, Context &ctx, AggregateContextPtr agg_context,
                                           size_t index)
    : SinkOp(exec, ctx), agg_context_(std::move(agg_context)), index_(index) {}

void AggregateBuildSinkOp::setPushedDownFilter(const std::string &pred, int op, Field constant) {
    has_filter_ = true;
    pred_ = pred;
    op_ = op;
    constant_ = constant;
}

// AggregateBuildSinkOp::writeImpl: the end-of-input block finishes this build task
OperatorStatus AggregateBuildSinkOp::writeImpl(Block &&block) {
    if (!block) {
        agg_context_->finishBuild(index_);
        return OperatorStatus::FINISHED;
    }
    if (has_filter_) agg_context_->buildOnBlockFiltered(index_, block, pred_, op_, constant_);
    else agg_context_->buildOnBlock(index_, block);
    return OperatorStatus::NEED_INPUT;
}

AggregateConvergentSourceOp::AggregateConvergentSourceOp(PipelineExecutorContext &exec, Context &ctx,
                                                         AggregateContextPtr agg_context, size_t index)
    : SourceOp(exec, ctx), agg_context_(std::move(agg_context)), index_(index) {
    setHeader(agg_context_->getHeader());
}

OperatorStatus AggregateConvergentSourceOp::readImpl(Block &block) {
    if (!agg_context_->allBuildFinished())
        throw Exception("convergent read before every build task finished", ErrorCodes::LOGICAL_ERROR);
    block = agg_context_->readForConvergent(index_);
    total_rows_ += block ? block.rows() : 0;
    return OperatorStatus::HAS_OUTPUT;
}

// ================================================================ hash join
JoinBuildContext::JoinBuildContext(Context &ctx, std::shared_ptr<Join> join, size_t build_concurrency,
                                   Block build_header)
    : ctx_(ctx), join_(std::move(join)), active_(std::max<size_t>(build_concurrency, 1)), build_header_(std::move(build_header)) {
    if (!join_) throw Exception("JoinBuildContext needs a Join", ErrorCodes::BAD_ARGUMENTS);
}

void JoinBuildContext::insertFromBlock(const Block &block) {
    std::lock_guard<std::mutex> g(mu_);
    if (finalized_) throw Exception("insertFromBlock after the build finished", ErrorCodes::LOGICAL_ERROR);
    join_->insertFromBlock(block);
    inserted_ = true;
}

bool JoinBuildContext::finishOneBuild() {
    std::lock_guard<std::mutex> g(mu_);
    if (active_ == 0) throw Exception("finishOneBuild called too often", ErrorCodes::LOGICAL_ERROR);
    if (--active_ > 0) return false;
    if (!inserted_) { // no build rows at all: an empty table of the build header's key types
        join_->initBuild(build_header_);
        join_->insertFromBlock(emptyLike(ctx_, build_header_));
    }
    join_->finishOneBuild();
    finalized_ = true;
    return true;
}

HashJoinBuildSink::HashJoinBuildSink(PipelineExecutorContext &exec, Context &ctx, JoinBuildContextPtr join,
                                     size_t op_index)
    : SinkOp(exec, ctx), join_(std::move(join)), op_index_(op_index) {}

OperatorStatus HashJoinBuildSink::writeImpl(Block &&block) {
    if (!block) {
        join_->finishOneBuild();
        return OperatorStatus::FINISHED;
    }
    join_->insertFromBlock(block);
    return OperatorStatus::NEED_INPUT;
}

HashJoinProbeTransformOp::HashJoinProbeTransformOp(PipelineExecutorContext &exec, Context &ctx,
                                                   JoinBuildContextPtr join, size_t op_index, size_t max_block_size)
    : TransformOp(exec, ctx), join_(std::move(join)), op_index_(op_index),
      max_block_size_(std::max<size_t>(max_block_size, 1)) {}

void HashJoinProbeTransformOp::transformHeaderImpl(Block &h) {
    if (!join_->isFinalized()) throw Exception("join should be finalized first", ErrorCodes::LOGICAL_ERROR);
    h = join_->join()->joinBlock(emptyLike(ctx_, h)).cloneEmpty();
}

OperatorStatus HashJoinProbeTransformOp::transformImpl(Block &block) {
    if (!join_->isFinalized()) throw Exception("join should be finalized first", ErrorCodes::LOGICAL_ERROR);
    if (!block) { // end of the probe side
        finished_ = true;
        return OperatorStatus::HAS_OUTPUT;
    }
    Block out = join_->join()->joinBlock(block);
    const size_t n = out ? out.rows() : 0;
    joined_rows_ += n;
    if (n == 0) return OperatorStatus::NEED_INPUT;
    if (n <= max_block_size_) {
        block = std::move(out);
        return OperatorStatus::HAS_OUTPUT;
    }
    for (size_t o = 0; o < n; o += max_block_size_) pending_.push_back(sliceBlock(ctx_, out, o, std::min(max_block_size_, n - o)));
    block = std::move(pending_.front());
    pending_.pop_front();
    return OperatorStatus::HAS_OUTPUT;
}

OperatorStatus HashJoinProbeTransformOp::tryOutputImpl(Block &block) {
    if (pending_.empty()) return OperatorStatus::NEED_INPUT;
    block = std::move(pending_.front());
    pending_.pop_front();
    return OperatorStatus::HAS_OUTPUT;
}

// ================================================================ exchange
void ExchangeReceiver::push(Block block, uint32_t stream) {
    std::lock_guard<std::mutex> g(mu_);
    queue_.emplace_back(stream, std::move(block));
}

void ExchangeReceiver::finish() { finished_ = true; }

bool ExchangeReceiver::tryPop(Block &block) {
    std::lock_guard<std::mutex> g(mu_);
    if (queue_.empty()) return false;
    block = std::move(queue_.front().second);
    queue_.pop_front();
    return true;
}

bool ExchangeReceiver::tryPop(Block &block, uint32_t stride, uint32_t index) {
    if (stride == 0) return tryPop(block);
    std::lock_guard<std::mutex> g(mu_);
    for (auto it = queue_.begin(); it != queue_.end(); ++it)
        if (it->first % stride == index) {
            block = std::move(it->second);
            queue_.erase(it);
            return true;
        }
    return false;
}

MPPTunnelSet::MPPTunnelSet(Context &ctx, uint32_t partition_num, size_t sender_concurrency, ExchangeReceiverPtr receiver,
                           MPPExchange *exchange, uint32_t local_partition, RemoteSink remote)
    : ctx_(ctx), partition_num_(partition_num), active_(std::max<size_t>(sender_concurrency, 1)),
      receiver_(std::move(receiver)), exchange_(exchange), local_partition_(local_partition), remote_(std::move(remote)),
      parts_(partition_num), streams_(partition_num) {
    if (partition_num == 0) throw Exception("partition_num must be positive", ErrorCodes::BAD_ARGUMENTS);
    if (exchange_ && (uint32_t)exchange_->nranks() != partition_num)
        throw Exception("an MPP exchange sends one partition per rank", ErrorCodes::BAD_ARGUMENTS);
    if (!exchange_ && local_partition_ >= partition_num)
        throw Exception("local partition out of range", ErrorCodes::BAD_ARGUMENTS);
}

void MPPTunnelSet::write(uint32_t part, Block &&block, uint32_t stream) {
    if (part >= partition_num_) throw Exception("partition out of range", ErrorCodes::BAD_ARGUMENTS);
    std::lock_guard<std::mutex> g(mu_);
    if (exchange_ && stream != 0) // the RCCL all-to-all moves one block per rank, without stream ids
        throw Exception("fine-grained shuffle over the RCCL exchange", ErrorCodes::NOT_IMPLEMENTED);
    if (!exchange_ && part != local_partition_) {
        if (remote_) remote_(part, std::move(block), stream);
        return;
    }
    parts_[part].push_back(std::move(block));
    streams_[part].push_back(stream);
}

void MPPTunnelSet::finishOneSender() {
    std::vector<std::vector<Block>> parts;
    std::vector<std::vector<uint32_t>> streams;
    {
        std::lock_guard<std::mutex> g(mu_);
        if (active_ == 0) throw Exception("finishOneSender called too often", ErrorCodes::LOGICAL_ERROR);
        if (--active_ > 0) return;
        parts.swap(parts_);
        streams.swap(streams_);
    }
    if (!exchange_) {
        for (size_t i = 0; i < parts[local_partition_].size(); ++i) {
            Block &b = parts[local_partition_][i];
            if (b && b.rows()) receiver_->push(std::move(b), streams[local_partition_][i]);
        }
        receiver_->finish();
        return;
    }
    // one block per destination rank (all-to-all; every rank calls this collectively)
    Block proto;
    for (auto &v : parts)
        for (auto &b : v)
            if (b && !proto) proto = b.cloneEmpty();
    if (!proto) throw Exception("MPP exchange without a block to take the schema from", ErrorCodes::LOGICAL_ERROR);
    std::vector<Block> send(partition_num_);
    for (uint32_t p = 0; p < partition_num_; ++p) {
        std::vector<Block> nonempty;
        for (Block &b : parts[p])
            if (b && b.rows()) nonempty.push_back(std::move(b));
        send[p] = nonempty.empty() ? emptyLike(ctx_, proto) : nonempty.size() == 1 ? nonempty[0] : concatenateBlocks(ctx_, nonempty);
    }
    Block got = exchange_->exchange(send);
    if (got && got.rows()) receiver_->push(std::move(got));
    receiver_->finish();
}

ExchangeSenderSinkOp::ExchangeSenderSinkOp(PipelineExecutorContext &exec, Context &ctx, MPPTunnelSetPtr tunnels,
                                           std::vector<size_t> partition_col_ids, std::vector<int> collators,
                                           int64_t batch_send_min_limit, uint32_t fine_grained_stream_count,
                                           uint64_t fine_grained_batch_size)
    : SinkOp(exec, ctx), tunnels_(std::move(tunnels)), partition_col_ids_(std::move(partition_col_ids)),
      collators_(std::move(collators)), limit_(batch_send_min_limit), fg_streams_(fine_grained_stream_count),
      fg_batch_(fine_grained_batch_size) {}

void ExchangeSenderSinkOp::operatePrefixImpl() {
    MPPTunnelSet *t = tunnels_.get();
    if (fg_streams_ > 0) { // each packet's chunks reach the tunnel as blocks tagged with their stream ids
        Context &ctx = ctx_;
        auto header = std::make_shared<Block>();
        fg_writer_ = std::make_unique<FineGrainedShuffleWriter>(
            ctx_, partition_col_ids_, t->partitionNum(), fg_streams_, fg_batch_,
            [t, &ctx, header](uint32_t part, FineGrainedPacket &&pk) {
                for (size_t i = 0; i < pk.chunks.size(); ++i)
                    t->write(part, CHBlockChunkCodecV1::decode(ctx, *header, pk.chunks[i]), pk.stream_ids[i]);
            });
        fg_header_ = header;
        fg_writer_->setCollators(collators_);
        return;
    }
    writer_ = std::make_unique<HashPartitionWriter>(
        ctx_, partition_col_ids_, t->partitionNum(), [t](uint32_t part, Block &&b) { t->write(part, std::move(b)); },
        limit_);
    writer_->setCollators(collators_);
}

// ExchangeSenderSinkOp::writeImpl: rows to the writer; the end-of-input block flushes
OperatorStatus ExchangeSenderSinkOp::writeImpl(Block &&block) {
    if (!writer_ && !fg_writer_) operatePrefixImpl();
    if (fg_writer_) {
        if (block) {
            if (!*fg_header_) *fg_header_ = block.cloneEmpty();
            total_rows_ += block.rows();
            fg_writer_->write(block);
            return OperatorStatus::NEED_INPUT;
        }
        fg_writer_->flush();
        tunnels_->finishOneSender();
        return OperatorStatus::FINISHED;
    }
    if (block) {
        total_rows_ += block.rows();
        writer_->write(block);
        return OperatorStatus::NEED_INPUT;
    }
    writer_->flush();
    tunnels_->finishOneSender();
    return OperatorStatus::FINISHED;
}

ExchangeReceiverSourceOp::ExchangeReceiverSourceOp(PipelineExecutorContext &exec, Context &ctx,
                                                   ExchangeReceiverPtr receiver, Block header, uint32_t stride,
                                                   uint32_t index)
    : SourceOp(exec, ctx), receiver_(std::move(receiver)), stride_(stride), index_(index) {
    setHeader(header.cloneEmpty());
}

OperatorStatus ExchangeReceiverSourceOp::readImpl(Block &block) {
    if (has_next_) {
        block = std::move(next_);
        has_next_ = false;
        return OperatorStatus::HAS_OUTPUT;
    }
    if (receiver_->tryPop(block, stride_, index_)) return OperatorStatus::HAS_OUTPUT;
    if (receiver_->finished()) { // drained after the last sender finished: end of input
        if (receiver_->tryPop(block, stride_, index_)) return OperatorStatus::HAS_OUTPUT;
        block = Block();
        return OperatorStatus::HAS_OUTPUT;
    }
    return OperatorStatus::WAITING;
}

OperatorStatus ExchangeReceiverSourceOp::awaitImpl() {
    if (!has_next_ && receiver_->tryPop(next_, stride_, index_)) has_next_ = true;
    return has_next_ || receiver_->finished() ? OperatorStatus::HAS_OUTPUT : OperatorStatus::WAITING;
}

// ================================================================ helpers
Block sliceBlock(Context &ctx, const Block &block, size_t offset, size_t rows) {
    const size_t n = block.rows();
    if (offset > n || rows > n - offset) throw Exception("slice out of range", ErrorCodes::BAD_ARGUMENTS);
    std::vector<uint32_t> perm(rows);
    for (size_t i = 0; i < rows; ++i) perm[i] = (uint32_t)(offset + i);
    DeviceBuffer dperm(ctx, std::max<size_t>(rows, 1) * 4);
    if (rows) check(tfg_upload(ctx.raw(), dperm.data(), perm.data(), rows * 4), "tfg_upload");
    Block out;
    for (const auto &c : block.getColumnsWithTypeAndName()) {
        ColumnPtr src = materialize(ctx, c.column);
        out.insert({gatherColumn(ctx, *src, (const uint32_t *)dperm.data(), rows, false), c.type, c.name});
    }
    ctx.sync();
    return out;
}

} // namespace tfa
