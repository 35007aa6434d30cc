// planner.h — executor descriptors -> operators: the step that instantiates the hot path's
// operators from a query plan (row b2 of SURVEY.md §8).
//
// The reference builds its operators from a tipb::Executor tree: PhysicalPlan::build
// (Flash/Planner/PhysicalPlan.cpp:95-231) turns each executor into a PhysicalPlanNode
// (TypeSelection :111, TypeAggregation :123, TypeExchangeSender :133, TypeExchangeReceiver :152,
// TypeJoin :204), the nodes split into pipelines at the pipeline breakers (aggregation build /
// convergent, join build / probe; PhysicalAggregation / PhysicalJoin::buildPipeline), and
// PipelineExecBuilder makes `concurrency` PipelineExecs of each pipeline.  The older stream
// engine (InterpreterDAG / DAGQueryBlockInterpreter) makes IBlockInputStream chains instead.
//
// tipb (contrib/tipb, unpinned) is absent from the reference copy, so the
// descriptor here is a repo-defined restatement of the tipb messages the path uses, with the
// same field names and meaning:
//   tipb::Expr          {tp, val (ColumnRef offset / literal), sig, children}
//   tipb::Executor      {tp, executor_id, selection.conditions, aggregation.group_by / agg_func,
//                        join.join_type / left_join_keys / right_join_keys / inner_idx /
//                        other_conditions, exchange_sender.tp / partition_keys,
//                        exchange_receiver.field_types, children}
// ColumnRef offsets index the child's output schema, as in tipb.  Output schemas follow TiDB's:
// Selection = its child's; Aggregation = the agg_func results, then the group_by columns
// (DAGExpressionAnalyzer::appendAggregation); Join = left columns then right columns (Semi /
// Anti: left only; LeftOuterSemi: left + the match helper); Projection = its exprs.
//
// MI355X-first choice: a Selection whose single condition is `column Op literal` directly under
// an Aggregation is pushed into the aggregation's build sink (the fused filter -> GROUP BY
// kernels, no mask materialised); PlanContext::fuse_filter_into_aggregation = false keeps the
// reference's FilterTransformOp -> AggregateBuildSinkOp shape.
#pragma once
#include <map>

#include "pipeline.h"

namespace tfa {
namespace dag {

enum class ExprType { ColumnRef, Int64, Uint64, Float64, MysqlDecimal, ScalarFunc, Sum, Count, Min, Max, First };

// the tipb::ScalarFuncSig values on the path (DAGUtils.cpp scalar_func_map names their functions)
enum class ScalarFuncSig {
    LTInt, LEInt, GTInt, GEInt, EQInt, NEInt,
    LTReal, LEReal, GTReal, GEReal, EQReal, NEReal,
    LTDecimal, LEDecimal, GTDecimal, GEDecimal, EQDecimal, NEDecimal,
    LogicalAnd, LogicalOr, UnaryNotInt,
    PlusInt, MinusInt, MultiplyInt, PlusReal, MinusReal, MultiplyReal, PlusDecimal, MinusDecimal, MultiplyDecimal,
};

struct Expr {
    ExprType tp = ExprType::ColumnRef;
    int64_t column = 0;         // ColumnRef: offset in the child's output schema
    Field literal;              // Int64 / Uint64 / Float64 / MysqlDecimal
    ScalarFuncSig sig = ScalarFuncSig::LTInt;
    std::vector<Expr> children; // ScalarFunc operands; aggregate arguments (count(*): none)
    int collator = TFG_COLLATOR_NONE; // field_type.collate of a min / max over a String (tfg_collator)

    static Expr col(int64_t offset);
    static Expr i64(int64_t v);
    static Expr u64(uint64_t v);
    static Expr f64(double v);
    static Expr decimal(int64_t raw, int scale);
    static Expr func(ScalarFuncSig sig, std::vector<Expr> args);
    static Expr sum(Expr arg);
    static Expr count();          // count(*)
    static Expr count(Expr arg);  // count(arg): non-NULL values
    // tipb::ExprType::Min / Max / First (first_row: TiDB's GROUP BY output columns, DAGUtils.cpp:69)
    static Expr min(Expr arg, int collator = TFG_COLLATOR_NONE);
    static Expr max(Expr arg, int collator = TFG_COLLATOR_NONE);
    static Expr firstRow(Expr arg);
};

enum class ExecType { TypeTableScan, TypeSelection, TypeAggregation, TypeJoin, TypeExchangeSender, TypeExchangeReceiver, TypeProjection };
enum class JoinType { TypeInnerJoin, TypeLeftOuterJoin, TypeRightOuterJoin, TypeSemiJoin, TypeAntiSemiJoin, TypeLeftOuterSemiJoin, TypeAntiLeftOuterSemiJoin };
enum class ExchangeType { PassThrough, Broadcast, Hash };

struct Executor {
    ExecType tp = ExecType::TypeTableScan;
    std::string executor_id;
    std::vector<Executor> children; // unary executors: one; TypeJoin: {left, right}
    // TypeTableScan (the mock table scan of executor tests): the PlanContext table of this name
    std::string table;
    // TypeSelection: ANDed conditions; TypeJoin: other_conditions over the joined schema
    std::vector<Expr> conditions;
    // TypeAggregation
    std::vector<Expr> group_by, agg_func;
    // TypeProjection
    std::vector<Expr> exprs;
    // TypeJoin
    JoinType join_type = JoinType::TypeInnerJoin;
    std::vector<Expr> left_join_keys, right_join_keys;
    int inner_idx = 1;              // the build side
    std::vector<int> join_collators; // tfg_collator per key (String keys); empty = binary
    // TypeExchangeSender
    ExchangeType exchange_type = ExchangeType::Hash;
    std::vector<Expr> partition_keys;
    std::vector<int> partition_collators;
    // tipb::Executor.fine_grained_shuffle_stream_count (ExchangeSender / ExchangeReceiver, > 0 =
    // fine-grained shuffle: a FineGrainedShuffleWriter on the sender, per-stream sources on the
    // receiver) and the batch size of a stream (the fine_grained_shuffle_batch_size setting)
    uint32_t fine_grained_shuffle_stream_count = 0;
    uint64_t fine_grained_shuffle_batch_size = 8192;
    // TypeExchangeReceiver: the PlanContext receiver of this name
    std::string receiver;

    static Executor tableScan(std::string id, std::string table);
    static Executor selection(std::string id, std::vector<Expr> conditions, Executor child);
    static Executor aggregation(std::string id, std::vector<Expr> group_by, std::vector<Expr> agg_func, Executor child);
    static Executor projection(std::string id, std::vector<Expr> exprs, Executor child);
    static Executor join(std::string id, JoinType type, std::vector<Expr> left_keys, std::vector<Expr> right_keys,
                         Executor left, Executor right, int inner_idx = 1);
    static Executor exchangeSender(std::string id, ExchangeType type, std::vector<Expr> partition_keys, Executor child);
    static Executor exchangeReceiver(std::string id, std::string receiver);
};

} // namespace dag

// What a plan reads and writes (the DAGContext / MPPTask's role): named table inputs, named
// exchange receivers, the sender's tunnels, the root's result handler, the concurrency.
struct PlanContext {
    struct Table {
        Block header;
        std::vector<Block> blocks;
    };
    struct Receiver {
        Block header;
        ExchangeReceiverPtr queue;
    };
    std::map<std::string, Table> tables;
    std::map<std::string, Receiver> receivers;
    MPPTunnelSetPtr tunnels;                   // TypeExchangeSender at the root
    GetResultSinkOp::ResultHandler result;     // any other root
    size_t concurrency = 2;                    // PipelineExecs per pipeline
    size_t max_block_size = 65536;             // join output slices
    bool fuse_filter_into_aggregation = true;  // see the header comment
};

// PhysicalPlan::build + buildPipeline + PipelineExecBuilder: pipelines in execution order (every
// pipeline after the ones it depends on), `concurrency` PipelineExecs each.
class PhysicalPlan {
public:
    PhysicalPlan(Context &ctx, PipelineExecutorContext &exec, PlanContext &env);
    ~PhysicalPlan();
    void build(const dag::Executor &root);
    std::vector<std::vector<PipelineExecPtr>> &pipelines() { return pipelines_; }
    Block outputHeader() const { return output_header_; }
    // runs every pipeline in order (runPipelineExecs); build() first
    void execute();
    // one line per pipeline: its operators' names, e.g. "BlocksSourceOp -> FilterTransformOp -> AggregateBuildSinkOp x2"
    std::string toString() const;

private:
    struct Stage;
    Context &ctx_;
    PipelineExecutorContext &exec_;
    PlanContext &env_;
    std::vector<std::vector<PipelineExecPtr>> pipelines_;
    Block output_header_;
    int tmp_ = 0;
    Stage lower(const dag::Executor &e);
    void applySelection(Stage &s, const dag::Executor &sel);
    void emit(Stage &s, const std::function<SinkOpPtr(size_t)> &sink);
};

// The stream engine's form of the same plan: an IBlockInputStream chain (the root's read()
// returns the result blocks; a TypeExchangeSender root writes its tunnels and passes blocks on).
BlockInputStreamPtr buildBlockInputStream(Context &ctx, PlanContext &env, const dag::Executor &root);

} // namespace tfa
