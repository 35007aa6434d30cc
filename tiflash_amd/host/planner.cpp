// planner.cpp — executor descriptors -> pipeline operators and IBlockInputStream chains (see
// planner.h for the reference map).
#include "planner.h"

#include <sstream>

namespace tfa {

// ================================================================ descriptor constructors
namespace dag {

Expr Expr::col(int64_t offset) {
    Expr e;
    e.tp = ExprType::ColumnRef;
    e.column = offset;
    return e;
}
Expr Expr::i64(int64_t v) {
    Expr e;
    e.tp = ExprType::Int64;
    e.literal = Field::Int64(v);
    return e;
}
Expr Expr::u64(uint64_t v) {
    Expr e;
    e.tp = ExprType::Uint64;
    e.literal = Field::UInt64(v);
    return e;
}
Expr Expr::f64(double v) {
    Expr e;
    e.tp = ExprType::Float64;
    e.literal = Field::Float64(v);
    return e;
}
Expr Expr::decimal(int64_t raw, int scale) {
    Expr e;
    e.tp = ExprType::MysqlDecimal;
    e.literal = Field::Decimal64(raw, scale);
    // a literal's precision is its digit count (TiDB types a decimal literal by its digits)
    uint64_t m = raw < 0 ? (uint64_t)(-(raw + 1)) + 1 : (uint64_t)raw;
    int digits = 1;
    while (m >= 10) {
        m /= 10;
        ++digits;
    }
    e.literal.prec = std::max(digits, scale + 1);
    return e;
}
Expr Expr::func(ScalarFuncSig sig, std::vector<Expr> args) {
    Expr e;
    e.tp = ExprType::ScalarFunc;
    e.sig = sig;
    e.children = std::move(args);
    return e;
}
Expr Expr::sum(Expr arg) {
    Expr e;
    e.tp = ExprType::Sum;
    e.children.push_back(std::move(arg));
    return e;
}
static Expr unaryAgg(ExprType tp, Expr arg) {
    Expr e;
    e.tp = tp;
    e.children.push_back(std::move(arg));
    return e;
}
Expr Expr::min(Expr arg, int collator) {
    Expr e = unaryAgg(ExprType::Min, std::move(arg));
    e.collator = collator;
    return e;
}
Expr Expr::max(Expr arg, int collator) {
    Expr e = unaryAgg(ExprType::Max, std::move(arg));
    e.collator = collator;
    return e;
}
Expr Expr::firstRow(Expr arg) { return unaryAgg(ExprType::First, std::move(arg)); }
Expr Expr::count() {
    Expr e;
    e.tp = ExprType::Count;
    return e;
}
Expr Expr::count(Expr arg) {
    Expr e;
    e.tp = ExprType::Count;
    e.children.push_back(std::move(arg));
    return e;
}

Executor Executor::tableScan(std::string id, std::string table) {
    Executor x;
    x.tp = ExecType::TypeTableScan;
    x.executor_id = std::move(id);
    x.table = std::move(table);
    return x;
}
Executor Executor::selection(std::string id, std::vector<Expr> conditions, Executor child) {
    Executor x;
    x.tp = ExecType::TypeSelection;
    x.executor_id = std::move(id);
    x.conditions = std::move(conditions);
    x.children.push_back(std::move(child));
    return x;
}
Executor Executor::aggregation(std::string id, std::vector<Expr> group_by, std::vector<Expr> agg_func, Executor child) {
    Executor x;
    x.tp = ExecType::TypeAggregation;
    x.executor_id = std::move(id);
    x.group_by = std::move(group_by);
    x.agg_func = std::move(agg_func);
    x.children.push_back(std::move(child));
    return x;
}
Executor Executor::projection(std::string id, std::vector<Expr> exprs, Executor child) {
    Executor x;
    x.tp = ExecType::TypeProjection;
    x.executor_id = std::move(id);
    x.exprs = std::move(exprs);
    x.children.push_back(std::move(child));
    return x;
}
Executor Executor::join(std::string id, JoinType type, std::vector<Expr> left_keys, std::vector<Expr> right_keys,
                        Executor left, Executor right, int inner_idx) {
    Executor x;
    x.tp = ExecType::TypeJoin;
    x.executor_id = std::move(id);
    x.join_type = type;
    x.left_join_keys = std::move(left_keys);
    x.right_join_keys = std::move(right_keys);
    x.inner_idx = inner_idx;
    x.children.push_back(std::move(left));
    x.children.push_back(std::move(right));
    return x;
}
Executor Executor::exchangeSender(std::string id, ExchangeType type, std::vector<Expr> partition_keys, Executor child) {
    Executor x;
    x.tp = ExecType::TypeExchangeSender;
    x.executor_id = std::move(id);
    x.exchange_type = type;
    x.partition_keys = std::move(partition_keys);
    x.children.push_back(std::move(child));
    return x;
}
Executor Executor::exchangeReceiver(std::string id, std::string receiver) {
    Executor x;
    x.tp = ExecType::TypeExchangeReceiver;
    x.executor_id = std::move(id);
    x.receiver = std::move(receiver);
    return x;
}

} // namespace dag

namespace {

using dag::ExecType;
using dag::Expr;
using dag::ExprType;
using dag::JoinType;
using dag::ScalarFuncSig;

[[noreturn]] void unsupported(const std::string &what) {
    throw Exception("plan: " + what + " is not supported on this path", ErrorCodes::NOT_IMPLEMENTED);
}

// scalar_func_map (Flash/Coprocessor/DAGUtils.cpp): comparison sigs -> tfg_cmp_op
bool compareOp(ScalarFuncSig s, int &op) {
    switch (s) {
    case ScalarFuncSig::LTInt: case ScalarFuncSig::LTReal: case ScalarFuncSig::LTDecimal: op = TFG_LT; return true;
    case ScalarFuncSig::LEInt: case ScalarFuncSig::LEReal: case ScalarFuncSig::LEDecimal: op = TFG_LE; return true;
    case ScalarFuncSig::GTInt: case ScalarFuncSig::GTReal: case ScalarFuncSig::GTDecimal: op = TFG_GT; return true;
    case ScalarFuncSig::GEInt: case ScalarFuncSig::GEReal: case ScalarFuncSig::GEDecimal: op = TFG_GE; return true;
    case ScalarFuncSig::EQInt: case ScalarFuncSig::EQReal: case ScalarFuncSig::EQDecimal: op = TFG_EQ; return true;
    case ScalarFuncSig::NEInt: case ScalarFuncSig::NEReal: case ScalarFuncSig::NEDecimal: op = TFG_NE; return true;
    default: return false;
    }
}
bool arithOp(ScalarFuncSig s, int &op) {
    switch (s) {
    case ScalarFuncSig::PlusInt: case ScalarFuncSig::PlusReal: case ScalarFuncSig::PlusDecimal: op = TFG_PLUS; return true;
    case ScalarFuncSig::MinusInt: case ScalarFuncSig::MinusReal: case ScalarFuncSig::MinusDecimal: op = TFG_MINUS; return true;
    case ScalarFuncSig::MultiplyInt: case ScalarFuncSig::MultiplyReal: case ScalarFuncSig::MultiplyDecimal:
        op = TFG_MULTIPLY;
        return true;
    default: return false;
    }
}
int swapCompare(int op) { // a Op b == b swap(Op) a
    switch (op) {
    case TFG_LT: return TFG_GT;
    case TFG_LE: return TFG_GE;
    case TFG_GT: return TFG_LT;
    case TFG_GE: return TFG_LE;
    default: return op;
    }
}
bool isLiteral(const Expr &e) {
    return e.tp == ExprType::Int64 || e.tp == ExprType::Uint64 || e.tp == ExprType::Float64 || e.tp == ExprType::MysqlDecimal;
}

const std::string &columnName(const Block &header, const Expr &e) {
    if (e.tp != ExprType::ColumnRef) unsupported("a non-ColumnRef expression where a column is expected");
    if (e.column < 0 || (size_t)e.column >= header.columns())
        throw Exception("ColumnRef " + std::to_string(e.column) + " out of the child's schema", ErrorCodes::BAD_ARGUMENTS);
    return header.safeGetByPosition((size_t)e.column).name;
}

// Appends the actions computing `e` over `header`'s columns (DAGExpressionAnalyzer::getActions)
// and returns the result column's name; ColumnRefs need no action.
std::string lowerExpr(ExpressionActions &ea, const Expr &e, const Block &header, const std::string &prefix, int &tmp) {
    if (e.tp == ExprType::ColumnRef) return columnName(header, e);
    if (e.tp != ExprType::ScalarFunc) unsupported("a literal or aggregate expression as a column");
    const std::string out = prefix + std::to_string(tmp++);
    int op = 0;
    if (compareOp(e.sig, op)) {
        if (e.children.size() != 2) throw Exception("comparison needs 2 operands", ErrorCodes::BAD_ARGUMENTS);
        const Expr &a = e.children[0], &b = e.children[1];
        if (isLiteral(b)) {
            ea.compare(lowerExpr(ea, a, header, prefix, tmp), op, b.literal, out);
        } else if (isLiteral(a)) {
            ea.compare(lowerExpr(ea, b, header, prefix, tmp), swapCompare(op), a.literal, out);
        } else {
            const std::string x = lowerExpr(ea, a, header, prefix, tmp), y = lowerExpr(ea, b, header, prefix, tmp);
            ea.compareColumns(x, op, y, out);
        }
        return out;
    }
    if (e.sig == ScalarFuncSig::LogicalAnd || e.sig == ScalarFuncSig::LogicalOr) {
        if (e.children.size() < 2) throw Exception("and / or needs >= 2 operands", ErrorCodes::BAD_ARGUMENTS);
        std::string acc = lowerExpr(ea, e.children[0], header, prefix, tmp);
        for (size_t i = 1; i < e.children.size(); ++i) {
            const std::string x = lowerExpr(ea, e.children[i], header, prefix, tmp);
            const std::string r = i + 1 == e.children.size() ? out : prefix + std::to_string(tmp++);
            ea.logical(e.sig == ScalarFuncSig::LogicalAnd ? TFG_AND : TFG_OR, acc, x, r);
            acc = r;
        }
        return out;
    }
    if (e.sig == ScalarFuncSig::UnaryNotInt) {
        if (e.children.size() != 1) throw Exception("not needs 1 operand", ErrorCodes::BAD_ARGUMENTS);
        ea.logical(TFG_NOT, lowerExpr(ea, e.children[0], header, prefix, tmp), "", out);
        return out;
    }
    if (arithOp(e.sig, op)) {
        if (e.children.size() != 2) throw Exception("arithmetic needs 2 operands", ErrorCodes::BAD_ARGUMENTS);
        const Expr &a = e.children[0], &b = e.children[1];
        if (isLiteral(a) && isLiteral(b)) unsupported("constant folding of two literals");
        if (isLiteral(b)) ea.arithmeticConst(op, lowerExpr(ea, a, header, prefix, tmp), b.literal, out);
        else if (isLiteral(a)) ea.arithmeticConstLeft(op, a.literal, lowerExpr(ea, b, header, prefix, tmp), out);
        else {
            const std::string x = lowerExpr(ea, a, header, prefix, tmp), y = lowerExpr(ea, b, header, prefix, tmp);
            ea.arithmetic(op, x, y, out);
        }
        return out;
    }
    unsupported("this scalar function");
}

// A transform keeping (and renaming) columns of its input: the Projection step the reference
// inserts after a filter (project_after_where), after an aggregation (the agg_func, group_by
// order of the schema) and around a join (buildFinalProjection's prefixed names).
class ProjectionTransformOp : public TransformOp {
public:
    ProjectionTransformOp(PipelineExecutorContext &exec, Context &ctx, std::vector<std::string> from,
                          std::vector<std::string> to)
        : TransformOp(exec, ctx), from_(std::move(from)), to_(std::move(to)) {}
    std::string getName() const override { return "ProjectionTransformOp"; }
    bool canHandleSelectiveBlock() const override { return true; }
    static Block project(const Block &in, const std::vector<std::string> &from, const std::vector<std::string> &to) {
        Block out;
        for (size_t i = 0; i < from.size(); ++i) {
            ColumnWithTypeAndName c = in.getByName(from[i]);
            c.name = to[i];
            out.insert(std::move(c));
        }
        out.info = in.info;
        return out;
    }

protected:
    OperatorStatus transformImpl(Block &block) override {
        if (block) block = project(block, from_, to_);
        return OperatorStatus::HAS_OUTPUT;
    }
    void transformHeaderImpl(Block &h) override { h = project(h, from_, to_); }

private:
    std::vector<std::string> from_, to_;
};

// ExchangeSender of type PassThrough (everything to tunnel 0) or Broadcast (every block to every
// tunnel) — Flash/Mpp/BroadcastOrPassThroughWriter.cpp
class BroadcastOrPassThroughSinkOp : public SinkOp {
public:
    BroadcastOrPassThroughSinkOp(PipelineExecutorContext &exec, Context &ctx, MPPTunnelSetPtr tunnels, bool broadcast)
        : SinkOp(exec, ctx), tunnels_(std::move(tunnels)), broadcast_(broadcast) {}
    std::string getName() const override { return broadcast_ ? "BroadcastSinkOp" : "PassThroughSinkOp"; }

protected:
    OperatorStatus writeImpl(Block &&block) override {
        if (!block) {
            tunnels_->finishOneSender();
            return OperatorStatus::FINISHED;
        }
        if (block.rows() == 0) return OperatorStatus::NEED_INPUT;
        if (!broadcast_) {
            tunnels_->write(0, std::move(block));
        } else {
            for (uint32_t p = 0; p < tunnels_->partitionNum(); ++p) {
                Block copy = block;
                tunnels_->write(p, std::move(copy));
            }
        }
        return OperatorStatus::NEED_INPUT;
    }

private:
    MPPTunnelSetPtr tunnels_;
    bool broadcast_;
};

std::vector<std::string> names(const Block &h) {
    std::vector<std::string> n;
    for (const auto &c : h.getColumnsWithTypeAndName()) n.push_back(c.name);
    return n;
}

Block renamedHeader(const Block &h, const std::string &prefix) {
    Block out;
    for (const auto &c : h.getColumnsWithTypeAndName()) out.insert({nullptr, c.type, prefix + c.name});
    return out;
}

// the Aggregator::Params of an aggregation executor over `header` (its group-by and argument
// expressions lowered into `pre` when they are not plain columns) and the agg_func output names
struct AggPlan {
    Aggregator::Params params;
    ExpressionActionsPtr pre; // null: every key / argument is a column
    std::vector<std::string> agg_names, key_names;
};
AggPlan planAggregation(Context &ctx, const dag::Executor &e, const Block &header) {
    AggPlan ap;
    auto ea = std::make_shared<ExpressionActions>(ctx);
    int tmp = 0;
    bool computed = false;
    const std::string prefix = e.executor_id + "_arg_";
    for (const Expr &k : e.group_by) {
        computed = computed || k.tp != ExprType::ColumnRef;
        ap.key_names.push_back(lowerExpr(*ea, k, header, prefix, tmp));
    }
    for (size_t i = 0; i < e.agg_func.size(); ++i) {
        const Expr &f = e.agg_func[i];
        AggregateDescription d;
        if (f.tp == ExprType::Sum) {
            if (f.children.size() != 1) throw Exception("sum needs one argument", ErrorCodes::BAD_ARGUMENTS);
            d.function = "sum";
        } else if (f.tp == ExprType::Count) {
            if (f.children.size() > 1) throw Exception("count takes at most one argument", ErrorCodes::BAD_ARGUMENTS);
            d.function = "count";
        } else if (f.tp == ExprType::Min || f.tp == ExprType::Max || f.tp == ExprType::First) {
            // AggregateFunctionMinMaxAny.cpp:155-159 (tipb Min / Max / First -> min / max / first_row,
            // DAGUtils.cpp:69)
            d.function = f.tp == ExprType::Min ? "min" : f.tp == ExprType::Max ? "max" : "first_row";
            d.collator = f.collator; // IAggregateFunction::setCollators (String min / max)
            if (f.children.size() != 1) throw Exception(d.function + " needs one argument", ErrorCodes::BAD_ARGUMENTS);
        } else {
            unsupported("this aggregate function");
        }
        for (const Expr &a : f.children) {
            computed = computed || a.tp != ExprType::ColumnRef;
            d.argument_names.push_back(lowerExpr(*ea, a, header, prefix, tmp));
        }
        d.column_name = e.executor_id + "_agg_" + std::to_string(i);
        ap.agg_names.push_back(d.column_name);
        ap.params.aggregates.push_back(d);
    }
    Block src = header;
    if (computed) {
        ap.pre = ea;
        Block z = emptyLike(ctx, header);
        ea->execute(z);
        src = z.cloneEmpty();
    }
    ap.params.src_header = src.cloneEmpty();
    ap.params.keys = ap.key_names;
    return ap;
}

// `Selection(col Op literal)` that can be pushed into the aggregation build (fused kernels)
bool pushableFilter(const dag::Executor &sel, const Block &header, std::string &col, int &op, Field &lit) {
    if (sel.tp != ExecType::TypeSelection || sel.conditions.size() != 1) return false;
    const Expr &c = sel.conditions[0];
    if (c.tp != ExprType::ScalarFunc || !compareOp(c.sig, op) || c.children.size() != 2) return false;
    const Expr &a = c.children[0], &b = c.children[1];
    if (a.tp == ExprType::ColumnRef && isLiteral(b)) {
        col = columnName(header, a);
        lit = b.literal;
        return true;
    }
    if (b.tp == ExprType::ColumnRef && isLiteral(a)) {
        col = columnName(header, b);
        lit = a.literal;
        op = swapCompare(op);
        return true;
    }
    return false;
}

JoinKind joinKind(JoinType t) {
    switch (t) {
    case JoinType::TypeInnerJoin: return JoinKind::Inner;
    case JoinType::TypeLeftOuterJoin: case JoinType::TypeRightOuterJoin: return JoinKind::Left;
    case JoinType::TypeSemiJoin: return JoinKind::Semi;
    case JoinType::TypeAntiSemiJoin: return JoinKind::Anti;
    case JoinType::TypeLeftOuterSemiJoin: return JoinKind::LeftOuterSemi;
    default: return JoinKind::AntiLeftOuterSemi;
    }
}

// the sides of a join executor: probe / build child index, checked against the join type
void joinSides(const dag::Executor &e, int &probe, int &build) {
    if (e.children.size() != 2) throw Exception("a join has two children", ErrorCodes::BAD_ARGUMENTS);
    if (e.inner_idx != 0 && e.inner_idx != 1) throw Exception("inner_idx must be 0 or 1", ErrorCodes::BAD_ARGUMENTS);
    build = e.inner_idx;
    probe = 1 - build;
    const bool right_build_only = e.join_type == JoinType::TypeLeftOuterJoin || e.join_type == JoinType::TypeSemiJoin ||
                                  e.join_type == JoinType::TypeAntiSemiJoin ||
                                  e.join_type == JoinType::TypeLeftOuterSemiJoin ||
                                  e.join_type == JoinType::TypeAntiLeftOuterSemiJoin;
    if (right_build_only && build != 1) unsupported("this join type with the left side as the build side");
    if (e.join_type == JoinType::TypeRightOuterJoin && build != 0)
        unsupported("a right outer join with the right side as the build side");
    if (e.left_join_keys.size() != e.right_join_keys.size() || e.left_join_keys.empty())
        throw Exception("join keys of both sides must pair up", ErrorCodes::BAD_ARGUMENTS);
}

// output header of joinBlock: probe columns, then the build columns (LEFT: nullable), or the
// probe columns alone (Semi / Anti), or + the match helper (LeftOuterSemi)
Block joinOutputHeader(JoinKind kind, const Block &probe, const Block &build, const std::string &helper) {
    Block out = probe.cloneEmpty();
    if (kind == JoinKind::Inner || kind == JoinKind::Left) {
        for (const auto &c : build.getColumnsWithTypeAndName()) {
            if (out.has(c.name)) continue;
            DataType t = c.type;
            if (kind == JoinKind::Left) t.nullable = true;
            out.insert({nullptr, t, c.name});
        }
    } else if (kind == JoinKind::LeftOuterSemi || kind == JoinKind::AntiLeftOuterSemi) {
        DataType i8;
        i8.type = TFG_INT8;
        i8.nullable = true;
        out.insert({nullptr, i8, helper});
    }
    return out;
}

// the joined schema in TiDB's order (left columns, then right ones) as names of the joinBlock output
std::vector<std::string> joinSchema(const dag::Executor &e, JoinKind kind, const Block &left, const Block &right,
                                    const std::string &helper) {
    std::vector<std::string> s = names(left);
    if (kind == JoinKind::Inner || kind == JoinKind::Left)
        for (const std::string &n : names(right)) s.push_back(n);
    if (kind == JoinKind::LeftOuterSemi || kind == JoinKind::AntiLeftOuterSemi) s.push_back(helper);
    (void)e;
    return s;
}

std::shared_ptr<Join> makeJoin(Context &ctx, const dag::Executor &e, const Block &probe_h, const Block &build_h,
                               const std::vector<std::string> &joined_schema, const Block &joined_header, int64_t expected) {
    int probe = 0, build = 1;
    joinSides(e, probe, build);
    const std::vector<Expr> &pk = probe == 0 ? e.left_join_keys : e.right_join_keys;
    const std::vector<Expr> &bk = probe == 0 ? e.right_join_keys : e.left_join_keys;
    std::vector<std::string> pn, bn;
    for (const Expr &k : pk) pn.push_back(columnName(probe_h, k));
    for (const Expr &k : bk) bn.push_back(columnName(build_h, k));
    auto join = std::make_shared<Join>(ctx, joinKind(e.join_type), pn, bn, expected, e.join_collators);
    if (!e.conditions.empty()) { // other_conditions over the joined schema (left then right)
        Block schema;
        for (const std::string &n : joined_schema) {
            const auto &c = joined_header.getByName(n);
            schema.insert({nullptr, c.type, n});
        }
        auto ea = std::make_shared<ExpressionActions>(ctx);
        int tmp = 0;
        std::string acc;
        for (size_t i = 0; i < e.conditions.size(); ++i) {
            const std::string r = lowerExpr(*ea, e.conditions[i], schema, e.executor_id + "_cond_", tmp);
            if (i == 0) {
                acc = r;
            } else {
                const std::string a = e.executor_id + "_cond_" + std::to_string(tmp++);
                ea->logical(TFG_AND, acc, r, a);
                acc = a;
            }
        }
        join->setOtherCondition(ea, acc);
    }
    return join;
}

} // namespace

// ================================================================ pipeline engine
struct PhysicalPlan::Stage {
    std::function<SourceOpPtr(size_t)> source;
    std::vector<std::function<TransformOpPtr(size_t)>> transforms;
    Block header;
    std::vector<std::string> ops; // operator names, for toString
    void project(PipelineExecutorContext &exec, Context &ctx, std::vector<std::string> from, std::vector<std::string> to) {
        header = ProjectionTransformOp::project(header, from, to);
        transforms.push_back([&exec, &ctx, from, to](size_t) -> TransformOpPtr {
            return std::make_unique<ProjectionTransformOp>(exec, ctx, from, to);
        });
        ops.push_back("ProjectionTransformOp");
    }
    void expression(PipelineExecutorContext &exec, Context &ctx, ExpressionActionsPtr ea) {
        Block z = emptyLike(ctx, header);
        ea->execute(z);
        header = z.cloneEmpty();
        transforms.push_back([&exec, &ctx, ea](size_t) -> TransformOpPtr {
            return std::make_unique<ExpressionTransformOp>(exec, ctx, ea);
        });
        ops.push_back("ExpressionTransformOp");
    }
};

PhysicalPlan::PhysicalPlan(Context &ctx, PipelineExecutorContext &exec, PlanContext &env)
    : ctx_(ctx), exec_(exec), env_(env) {}
PhysicalPlan::~PhysicalPlan() = default;

void PhysicalPlan::emit(Stage &s, const std::function<SinkOpPtr(size_t)> &sink) {
    std::vector<PipelineExecPtr> execs;
    for (size_t i = 0; i < env_.concurrency; ++i) {
        TransformOps tr;
        for (auto &f : s.transforms) tr.push_back(f(i));
        execs.push_back(std::make_unique<PipelineExec>(s.source(i), std::move(tr), sink(i)));
    }
    pipelines_.push_back(std::move(execs));
}

// FilterTransformOp over the ANDed conditions, then project_after_where (the child's schema)
void PhysicalPlan::applySelection(Stage &s, const dag::Executor &e) {
    if (e.conditions.empty()) return;
    PipelineExecutorContext &exec = exec_;
    Context &ctx = ctx_;
    const std::vector<std::string> keep = names(s.header);
    auto ea = std::make_shared<ExpressionActions>(ctx);
    std::string acc;
    for (size_t i = 0; i < e.conditions.size(); ++i) {
        const std::string r = lowerExpr(*ea, e.conditions[i], s.header, e.executor_id + "_", tmp_);
        if (i == 0) {
            acc = r;
        } else {
            const std::string a = e.executor_id + "_" + std::to_string(tmp_++);
            ea->logical(TFG_AND, acc, r, a);
            acc = a;
        }
    }
    const Block in = s.header;
    const std::string fcol = acc;
    s.transforms.push_back([&exec, &ctx, in, ea, fcol](size_t) -> TransformOpPtr {
        return std::make_unique<FilterTransformOp>(exec, ctx, in, ea, fcol);
    });
    s.ops.push_back("FilterTransformOp");
    Block z = emptyLike(ctx, in);
    ea->execute(z);
    s.header = z.cloneEmpty();
    s.project(exec, ctx, keep, keep);
}

PhysicalPlan::Stage PhysicalPlan::lower(const dag::Executor &e) {
    const size_t conc = std::max<size_t>(env_.concurrency, 1);
    PipelineExecutorContext &exec = exec_;
    Context &ctx = ctx_;
    auto unary = [&]() -> const dag::Executor & {
        if (e.children.size() != 1) throw Exception(e.executor_id + ": needs one child", ErrorCodes::BAD_ARGUMENTS);
        return e.children[0];
    };
    switch (e.tp) {
    case ExecType::TypeTableScan: {
        auto it = env_.tables.find(e.table);
        if (it == env_.tables.end()) throw Exception("plan: no table " + e.table, ErrorCodes::BAD_ARGUMENTS);
        const PlanContext::Table &t = it->second;
        Stage s;
        s.header = t.header ? t.header.cloneEmpty() : (t.blocks.empty() ? Block() : t.blocks[0].cloneEmpty());
        const Block h = s.header;
        const std::vector<Block> *blocks = &t.blocks;
        s.source = [&exec, &ctx, h, blocks, conc](size_t i) -> SourceOpPtr {
            std::vector<Block> mine;
            for (size_t b = i; b < blocks->size(); b += conc) mine.push_back((*blocks)[b]);
            return std::make_unique<BlocksSourceOp>(exec, ctx, h, std::move(mine));
        };
        s.ops.push_back("BlocksSourceOp");
        return s;
    }
    case ExecType::TypeExchangeReceiver: {
        auto it = env_.receivers.find(e.receiver);
        if (it == env_.receivers.end()) throw Exception("plan: no receiver " + e.receiver, ErrorCodes::BAD_ARGUMENTS);
        Stage s;
        s.header = it->second.header.cloneEmpty();
        const Block h = s.header;
        ExchangeReceiverPtr q = it->second.queue;
        // fine-grained shuffle: PipelineExec i reads the streams s with s % concurrency == i
        const uint32_t stride = e.fine_grained_shuffle_stream_count ? (uint32_t)std::max<size_t>(env_.concurrency, 1) : 0;
        s.source = [&exec, &ctx, h, q, stride](size_t i) -> SourceOpPtr {
            return std::make_unique<ExchangeReceiverSourceOp>(exec, ctx, q, h, stride, stride ? (uint32_t)i : 0);
        };
        s.ops.push_back("ExchangeReceiverSourceOp");
        return s;
    }
    case ExecType::TypeSelection: {
        Stage s = lower(unary());
        applySelection(s, e);
        return s;
    }
    case ExecType::TypeProjection: {
        Stage s = lower(unary());
        auto ea = std::make_shared<ExpressionActions>(ctx);
        std::vector<std::string> from, to;
        bool computed = false;
        for (size_t i = 0; i < e.exprs.size(); ++i) {
            computed = computed || e.exprs[i].tp != ExprType::ColumnRef;
            from.push_back(lowerExpr(*ea, e.exprs[i], s.header, e.executor_id + "_", tmp_));
            to.push_back(e.executor_id + "_" + std::to_string(i) + (e.exprs[i].tp == ExprType::ColumnRef ? "_" + from.back() : ""));
        }
        if (computed) s.expression(exec, ctx, ea);
        s.project(exec, ctx, from, to);
        return s;
    }
    case ExecType::TypeAggregation: {
        const dag::Executor &child = unary();
        // a `col Op literal` Selection right below goes into the build sink (fused kernels)
        std::string pcol;
        int pop = 0;
        Field plit;
        bool pushed = false;
        Stage s;
        if (env_.fuse_filter_into_aggregation && child.tp == ExecType::TypeSelection && child.children.size() == 1) {
            s = lower(child.children[0]); // lowered once: its pipelines are emitted once
            pushed = pushableFilter(child, s.header, pcol, pop, plit);
            if (!pushed) applySelection(s, child);
        } else {
            s = lower(child);
        }
        AggPlan ap = planAggregation(ctx, e, s.header);
        if (ap.pre) s.expression(exec, ctx, ap.pre);
        auto agg_ctx = std::make_shared<AggregateContext>(ctx, ap.params, conc);
        emit(s, [&exec, &ctx, agg_ctx, pushed, pcol, pop, plit](size_t i) -> SinkOpPtr {
            auto sink = std::make_unique<AggregateBuildSinkOp>(exec, ctx, agg_ctx, i);
            if (pushed) sink->setPushedDownFilter(pcol, pop, plit);
            return sink;
        });
        Stage out;
        out.header = agg_ctx->getHeader();
        out.source = [&exec, &ctx, agg_ctx](size_t i) -> SourceOpPtr {
            return std::make_unique<AggregateConvergentSourceOp>(exec, ctx, agg_ctx, i);
        };
        out.ops.push_back("AggregateConvergentSourceOp");
        // schema: the agg_func results, then the group-by columns
        std::vector<std::string> order = ap.agg_names;
        for (const std::string &k : ap.key_names) order.push_back(k);
        out.project(exec, ctx, order, order);
        return out;
    }
    case ExecType::TypeJoin: {
        int probe = 0, build = 1;
        joinSides(e, probe, build);
        const JoinKind kind = joinKind(e.join_type);
        // buildFinalProjection of both sides: prefixed names, so no column name repeats
        Stage sb = lower(e.children[build]);
        const std::string bpre = e.executor_id + (build == 0 ? "_l_" : "_r_");
        sb.project(exec, ctx, names(sb.header), names(renamedHeader(sb.header, bpre)));
        Stage sp = lower(e.children[probe]);
        const std::string ppre = e.executor_id + (probe == 0 ? "_l_" : "_r_");
        sp.project(exec, ctx, names(sp.header), names(renamedHeader(sp.header, ppre)));
        const std::string helper = e.executor_id + "_match_helper";
        const Block out_h = joinOutputHeader(kind, sp.header, sb.header, helper);
        const Block &left = probe == 0 ? sp.header : sb.header, &right = probe == 0 ? sb.header : sp.header;
        const std::vector<std::string> schema = joinSchema(e, kind, left, right, helper);
        auto join = makeJoin(ctx, e, sp.header, sb.header, schema, out_h, 0);
        join->setMatchHelperName(helper);
        auto jctx = std::make_shared<JoinBuildContext>(ctx, join, conc, sb.header);
        emit(sb, [&exec, &ctx, jctx](size_t i) -> SinkOpPtr { return std::make_unique<HashJoinBuildSink>(exec, ctx, jctx, i); });
        const size_t mbs = env_.max_block_size;
        sp.transforms.push_back([&exec, &ctx, jctx, mbs](size_t i) -> TransformOpPtr {
            return std::make_unique<HashJoinProbeTransformOp>(exec, ctx, jctx, i, mbs);
        });
        sp.ops.push_back("HashJoinProbeTransformOp");
        sp.header = out_h;
        sp.project(exec, ctx, schema, schema);
        return sp;
    }
    case ExecType::TypeExchangeSender:
        unsupported("an ExchangeSender below the root");
    }
    unsupported("this executor type");
}

void PhysicalPlan::build(const dag::Executor &root) {
    pipelines_.clear();
    PipelineExecutorContext &exec = exec_;
    Context &ctx = ctx_;
    if (root.tp == ExecType::TypeExchangeSender) {
        if (root.children.size() != 1) throw Exception("ExchangeSender needs one child", ErrorCodes::BAD_ARGUMENTS);
        if (!env_.tunnels) throw Exception("plan: an ExchangeSender root needs PlanContext::tunnels", ErrorCodes::BAD_ARGUMENTS);
        Stage s = lower(root.children[0]);
        output_header_ = s.header;
        MPPTunnelSetPtr tunnels = env_.tunnels;
        if (root.exchange_type == dag::ExchangeType::Hash) {
            std::vector<size_t> ids;
            for (const Expr &k : root.partition_keys) {
                if (k.tp != ExprType::ColumnRef || k.column < 0 || (size_t)k.column >= s.header.columns())
                    throw Exception("partition keys are ColumnRefs of the child's schema", ErrorCodes::BAD_ARGUMENTS);
                ids.push_back((size_t)k.column);
            }
            std::vector<int> coll = root.partition_collators;
            const uint32_t fgs = root.fine_grained_shuffle_stream_count;
            const uint64_t fgb = root.fine_grained_shuffle_batch_size;
            emit(s, [&exec, &ctx, tunnels, ids, coll, fgs, fgb](size_t) -> SinkOpPtr {
                return std::make_unique<ExchangeSenderSinkOp>(exec, ctx, tunnels, ids, coll, -1, fgs, fgb);
            });
        } else {
            const bool bc = root.exchange_type == dag::ExchangeType::Broadcast;
            emit(s, [&exec, &ctx, tunnels, bc](size_t) -> SinkOpPtr {
                return std::make_unique<BroadcastOrPassThroughSinkOp>(exec, ctx, tunnels, bc);
            });
        }
        return;
    }
    Stage s = lower(root);
    output_header_ = s.header;
    auto handler = env_.result;
    if (!handler) throw Exception("plan: the root needs PlanContext::result", ErrorCodes::BAD_ARGUMENTS);
    emit(s, [&exec, &ctx, handler](size_t) -> SinkOpPtr { return std::make_unique<GetResultSinkOp>(exec, ctx, handler); });
}

void PhysicalPlan::execute() {
    for (auto &p : pipelines_) runPipelineExecs(exec_, p);
}

std::string PhysicalPlan::toString() const {
    std::ostringstream os;
    for (const auto &p : pipelines_) {
        if (p.empty()) continue;
        const PipelineExec &pe = *p[0];
        os << pe.source().getName();
        for (const auto &t : pe.transforms()) os << " -> " << t->getName();
        os << " -> " << pe.sink().getName() << " x" << p.size() << "\n";
    }
    return os.str();
}

// ================================================================ stream engine
namespace {

class ProjectionBlockInputStream : public IBlockInputStream {
public:
    // in_header: the input's structure when its stream cannot tell (a join's probe stream
    // reports its probe header)
    ProjectionBlockInputStream(BlockInputStreamPtr in, std::vector<std::string> from, std::vector<std::string> to,
                               Block in_header = Block())
        : in_(std::move(in)), from_(std::move(from)), to_(std::move(to)), in_header_(std::move(in_header)) {}
    std::string getName() const override { return "Projection"; }
    Block getHeader() const override {
        return ProjectionTransformOp::project(in_header_ ? in_header_ : in_->getHeader(), from_, to_);
    }
    Block read() override {
        Block b = in_->read();
        return b ? ProjectionTransformOp::project(b, from_, to_) : b;
    }

private:
    BlockInputStreamPtr in_;
    std::vector<std::string> from_, to_;
    Block in_header_;
};

class ExpressionBlockInputStream : public IBlockInputStream {
public:
    ExpressionBlockInputStream(Context &ctx, BlockInputStreamPtr in, ExpressionActionsPtr ea)
        : ctx_(ctx), in_(std::move(in)), ea_(std::move(ea)) {}
    std::string getName() const override { return "Expression"; }
    Block getHeader() const override {
        Block z = emptyLike(ctx_, in_->getHeader());
        ea_->execute(z);
        return z.cloneEmpty();
    }
    Block read() override {
        Block b = in_->read();
        if (b) ea_->execute(b);
        return b;
    }

private:
    Context &ctx_;
    BlockInputStreamPtr in_;
    ExpressionActionsPtr ea_;
};

class ExchangeReceiverInputStream : public IBlockInputStream {
public:
    ExchangeReceiverInputStream(ExchangeReceiverPtr q, Block header) : q_(std::move(q)), header_(std::move(header)) {}
    std::string getName() const override { return "ExchangeReceiver"; }
    Block getHeader() const override { return header_; }
    Block read() override {
        Block b;
        for (;;) {
            if (q_->tryPop(b)) {
                if (b && b.rows()) return b;
                continue;
            }
            if (q_->finished()) {
                if (q_->tryPop(b)) {
                    if (b && b.rows()) return b;
                    continue;
                }
                return Block();
            }
            throw Exception("ExchangeReceiver stream: no block queued and the senders are not finished",
                            ErrorCodes::LOGICAL_ERROR);
        }
    }

private:
    ExchangeReceiverPtr q_;
    Block header_;
};

// ExchangeSenderBlockInputStream (DataStreams/ExchangeSenderBlockInputStream.cpp): every block
// read goes to the writer and is passed on; the end of input flushes and finishes the sender
class ExchangeSenderBlockInputStream : public IBlockInputStream {
public:
    ExchangeSenderBlockInputStream(Context &ctx, BlockInputStreamPtr in, MPPTunnelSetPtr tunnels, dag::ExchangeType type,
                                   std::vector<size_t> ids, std::vector<int> collators)
        : in_(std::move(in)), tunnels_(std::move(tunnels)), type_(type) {
        if (type_ == dag::ExchangeType::Hash) {
            MPPTunnelSet *t = tunnels_.get();
            writer_ = std::make_unique<HashPartitionWriter>(
                ctx, std::move(ids), t->partitionNum(), [t](uint32_t part, Block &&b) { t->write(part, std::move(b)); });
            writer_->setCollators(std::move(collators));
        }
    }
    std::string getName() const override { return "ExchangeSender"; }
    Block getHeader() const override { return in_->getHeader(); }
    Block read() override {
        Block b = in_->read();
        if (!b) {
            if (!done_) {
                if (writer_) writer_->flush();
                tunnels_->finishOneSender();
                done_ = true;
            }
            return b;
        }
        if (writer_) {
            writer_->write(b);
        } else if (b.rows()) {
            for (uint32_t p = 0; p < (type_ == dag::ExchangeType::Broadcast ? tunnels_->partitionNum() : 1u); ++p) {
                Block copy = b;
                tunnels_->write(p, std::move(copy));
            }
        }
        return b;
    }

private:
    BlockInputStreamPtr in_;
    MPPTunnelSetPtr tunnels_;
    dag::ExchangeType type_;
    std::unique_ptr<HashPartitionWriter> writer_;
    bool done_ = false;
};

BlockInputStreamPtr lowerStream(Context &ctx, PlanContext &env, const dag::Executor &e, int &tmp) {
    auto unary = [&]() -> const dag::Executor & {
        if (e.children.size() != 1) throw Exception(e.executor_id + ": needs one child", ErrorCodes::BAD_ARGUMENTS);
        return e.children[0];
    };
    switch (e.tp) {
    case ExecType::TypeTableScan: {
        auto it = env.tables.find(e.table);
        if (it == env.tables.end()) throw Exception("plan: no table " + e.table, ErrorCodes::BAD_ARGUMENTS);
        return std::make_shared<BlocksListBlockInputStream>(it->second.blocks);
    }
    case ExecType::TypeExchangeReceiver: {
        auto it = env.receivers.find(e.receiver);
        if (it == env.receivers.end()) throw Exception("plan: no receiver " + e.receiver, ErrorCodes::BAD_ARGUMENTS);
        return std::make_shared<ExchangeReceiverInputStream>(it->second.queue, it->second.header.cloneEmpty());
    }
    case ExecType::TypeSelection: {
        BlockInputStreamPtr in = lowerStream(ctx, env, unary(), tmp);
        if (e.conditions.empty()) return in;
        const Block h = in->getHeader();
        auto ea = std::make_shared<ExpressionActions>(ctx);
        std::string acc;
        for (size_t i = 0; i < e.conditions.size(); ++i) {
            const std::string r = lowerExpr(*ea, e.conditions[i], h, e.executor_id + "_", tmp);
            if (i == 0) {
                acc = r;
            } else {
                const std::string a = e.executor_id + "_" + std::to_string(tmp++);
                ea->logical(TFG_AND, acc, r, a);
                acc = a;
            }
        }
        BlockInputStreamPtr f = std::make_shared<FilterBlockInputStream>(ctx, in, ea, acc);
        return std::make_shared<ProjectionBlockInputStream>(f, names(h), names(h));
    }
    case ExecType::TypeProjection: {
        BlockInputStreamPtr in = lowerStream(ctx, env, unary(), tmp);
        const Block h = in->getHeader();
        auto ea = std::make_shared<ExpressionActions>(ctx);
        std::vector<std::string> from, to;
        bool computed = false;
        for (size_t i = 0; i < e.exprs.size(); ++i) {
            computed = computed || e.exprs[i].tp != ExprType::ColumnRef;
            from.push_back(lowerExpr(*ea, e.exprs[i], h, e.executor_id + "_", tmp));
            to.push_back(e.executor_id + "_" + std::to_string(i) + (e.exprs[i].tp == ExprType::ColumnRef ? "_" + from.back() : ""));
        }
        if (computed) in = std::make_shared<ExpressionBlockInputStream>(ctx, in, ea);
        return std::make_shared<ProjectionBlockInputStream>(in, from, to);
    }
    case ExecType::TypeAggregation: {
        BlockInputStreamPtr in = lowerStream(ctx, env, unary(), tmp);
        AggPlan ap = planAggregation(ctx, e, in->getHeader());
        if (ap.pre) in = std::make_shared<ExpressionBlockInputStream>(ctx, in, ap.pre);
        BlockInputStreamPtr agg = std::make_shared<AggregatingBlockInputStream>(ctx, in, ap.params);
        std::vector<std::string> order = ap.agg_names;
        for (const std::string &k : ap.key_names) order.push_back(k);
        return std::make_shared<ProjectionBlockInputStream>(agg, order, order);
    }
    case ExecType::TypeJoin: {
        int probe = 0, build = 1;
        joinSides(e, probe, build);
        const JoinKind kind = joinKind(e.join_type);
        BlockInputStreamPtr bs = lowerStream(ctx, env, e.children[build], tmp);
        const Block bh0 = bs->getHeader();
        const Block bh = renamedHeader(bh0, e.executor_id + (build == 0 ? "_l_" : "_r_"));
        bs = std::make_shared<ProjectionBlockInputStream>(bs, names(bh0), names(bh));
        BlockInputStreamPtr ps = lowerStream(ctx, env, e.children[probe], tmp);
        const Block ph0 = ps->getHeader();
        const Block ph = renamedHeader(ph0, e.executor_id + (probe == 0 ? "_l_" : "_r_"));
        ps = std::make_shared<ProjectionBlockInputStream>(ps, names(ph0), names(ph));
        const std::string helper = e.executor_id + "_match_helper";
        const Block out_h = joinOutputHeader(kind, ph, bh, helper);
        const Block &left = probe == 0 ? ph : bh, &right = probe == 0 ? bh : ph;
        const std::vector<std::string> schema = joinSchema(e, kind, left, right, helper);
        auto join = makeJoin(ctx, e, ph, bh, schema, out_h, 0);
        join->setMatchHelperName(helper);
        // the build side is read to the end first (HashJoinBuildBlockInputStream), then probed
        join->initBuild(bh);
        bool any = false;
        for (Block b = bs->read(); b; b = bs->read()) {
            join->insertFromBlock(b);
            any = true;
        }
        if (!any) join->insertFromBlock(emptyLike(ctx, bh));
        join->finishOneBuild();
        BlockInputStreamPtr probe_s = std::make_shared<HashJoinProbeBlockInputStream>(ps, join);
        return std::make_shared<ProjectionBlockInputStream>(probe_s, schema, schema, out_h);
    }
    case ExecType::TypeExchangeSender: {
        BlockInputStreamPtr in = lowerStream(ctx, env, unary(), tmp);
        if (!env.tunnels) throw Exception("plan: an ExchangeSender needs PlanContext::tunnels", ErrorCodes::BAD_ARGUMENTS);
        std::vector<size_t> ids;
        for (const Expr &k : e.partition_keys) ids.push_back((size_t)k.column);
        return std::make_shared<ExchangeSenderBlockInputStream>(ctx, in, env.tunnels, e.exchange_type, ids,
                                                                e.partition_collators);
    }
    }
    unsupported("this executor type");
}

} // namespace

BlockInputStreamPtr buildBlockInputStream(Context &ctx, PlanContext &env, const dag::Executor &root) {
    int tmp = 0;
    return lowerStream(ctx, env, root, tmp);
}

} // namespace tfa
