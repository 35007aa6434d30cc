// filter.cpp — ExpressionActions (a1-a4) and FilterTransformAction (a5-a8) over the C-ABI.
#include <algorithm>
#include <cstring>

#include "tfa_host.h"

namespace tfa {

Field Field::Int64(int64_t v) {
    Field f;
    f.type = TFG_INT64;
    memcpy(&f.bits, &v, 8);
    return f;
}
Field Field::UInt64(uint64_t v) {
    Field f;
    f.type = TFG_UINT64;
    f.bits = v;
    return f;
}
Field Field::Float64(double v) {
    Field f;
    f.type = TFG_FLOAT64;
    memcpy(&f.bits, &v, 8);
    return f;
}
Field Field::Decimal64(int64_t raw, int scale) {
    Field f;
    f.type = TFG_DECIMAL64;
    memcpy(&f.bits, &raw, 8);
    f.scale = scale;
    return f;
}

ExpressionActions &ExpressionActions::compare(const std::string &lhs, int op, Field constant, const std::string &result) {
    actions_.push_back({0, op, lhs, "", result, constant});
    return *this;
}
ExpressionActions &ExpressionActions::compareColumns(const std::string &lhs, int op, const std::string &rhs,
                                                     const std::string &result) {
    actions_.push_back({1, op, lhs, rhs, result, Field{}});
    return *this;
}
ExpressionActions &ExpressionActions::logical(int op, const std::string &a, const std::string &b, const std::string &result) {
    actions_.push_back({2, op, a, b, result, Field{}});
    return *this;
}
ExpressionActions &ExpressionActions::arithmetic(int op, const std::string &a, const std::string &b, const std::string &result) {
    actions_.push_back({3, op, a, b, result, Field{}});
    return *this;
}
ExpressionActions &ExpressionActions::arithmeticConst(int op, const std::string &a, Field b, const std::string &result) {
    actions_.push_back({4, op, a, "", result, b});
    return *this;
}
ExpressionActions &ExpressionActions::arithmeticConstLeft(int op, Field a, const std::string &b, const std::string &result) {
    actions_.push_back({5, op, "", b, result, a});
    return *this;
}

bool ExpressionActions::singleCompare(std::string &column, int &op, Field &constant, std::string &result) const {
    if (actions_.size() != 1 || actions_[0].kind != 0) return false;
    column = actions_[0].a;
    op = actions_[0].op;
    constant = actions_[0].constant;
    result = actions_[0].result;
    return true;
}

namespace {

bool isDecimal(int t) { return t == TFG_DECIMAL32 || t == TFG_DECIMAL64 || t == TFG_DECIMAL128 || t == TFG_DECIMAL256; }

// IntPrec<T>::prec (Common/Decimal.h:45-93): an integer operand of decimal arithmetic is
// Decimal(IntPrec, 0)
int intPrec(int t) {
    switch (t) {
    case TFG_INT8: case TFG_UINT8: return 3;
    case TFG_INT16: case TFG_UINT16: return 5;
    case TFG_INT32: case TFG_UINT32: return 10;
    case TFG_INT64: return 19;
    default: return 20; // UInt64
    }
}
bool isFloat(int t) { return t == TFG_FLOAT32 || t == TFG_FLOAT64; }
bool isUnsigned(int t) { return t >= TFG_UINT8 && t <= TFG_UINT64; }

// result type of a +|-|* b (FunctionBinaryArithmetic result-type rules restricted to the path:
// integers -> 64-bit of the operands' signedness, floats -> Float64; decimals by the inferers of
// Common/Decimal.h:109-163 — PlusDecimalInferer: scale max(s1, s2), precision
// min(max(p1 - s1, p2 - s2) + scale + 1, 65); MulDecimalInferer: (min(p1 + p2, 65), min(s1 + s2, 30))
// — stored in the narrowest Decimal of that precision (createDecimal)
DataType arithResult(int op, const DataType &a, const DataType &b) {
    DataType r;
    r.nullable = a.nullable || b.nullable;
    if (isDecimal(a.type) || isDecimal(b.type)) {
        if (isFloat(a.type) || isFloat(b.type))
            throw Exception("decimal arithmetic with a float operand", ErrorCodes::ILLEGAL_TYPE_OF_ARGUMENT);
        const int sa = isDecimal(a.type) ? a.scale : 0, sb = isDecimal(b.type) ? b.scale : 0;
        const int pa = isDecimal(a.type) ? a.precision() : intPrec(a.type);
        const int pb = isDecimal(b.type) ? b.precision() : intPrec(b.type);
        int prec, scale;
        if (op == TFG_MULTIPLY) {
            prec = std::min(pa + pb, 65);
            scale = std::min(sa + sb, 30);
        } else {
            scale = std::max(sa, sb);
            prec = std::min(std::max(pa - sa, pb - sb) + scale + 1, 65);
        }
        return DataType::decimal(prec, scale, r.nullable); // Decimal256 past precision 38
    }
    if (isFloat(a.type) || isFloat(b.type)) {
        r.type = TFG_FLOAT64;
        return r;
    }
    r.type = (isUnsigned(a.type) && isUnsigned(b.type)) ? TFG_UINT64 : TFG_INT64;
    return r;
}

ColumnPtr newColumn(Context &ctx, DataType type, size_t rows) {
    auto c = std::make_shared<IColumn>();
    c->type = type;
    c->type.nullable = false;
    c->rows = rows;
    c->data = std::make_shared<DeviceBuffer>(ctx, rows * std::max<size_t>(type.width(), 1));
    return c;
}

// OR of two optional null maps into a fresh buffer (default NULL handling of IFunction)
DeviceBufferPtr mergeNulls(Context &ctx, const IColumn &a, const IColumn *b, size_t n) {
    const uint8_t *na = a.nullPtr(), *nb = b ? b->nullPtr() : nullptr;
    if (!na && !nb) return nullptr;
    auto out = std::make_shared<DeviceBuffer>(ctx, n);
    if (na && nb)
        check(tfg_mask_logic(ctx.raw(), TFG_OR, na, nb, (int64_t)n, (uint8_t *)out->data()), "tfg_mask_logic");
    else
        check(tfg_copy(ctx.raw(), out->data(), na ? na : nb, n), "tfg_copy");
    return out;
}

} // namespace

void ExpressionActions::execute(Block &block) const {
    const size_t n = block.rows();
    for (const Action &act : actions_) {
        ColumnPtr res;
        DataType rt;
        rt.type = TFG_UINT8;
        switch (act.kind) {
        case 0: { // column Op constant: NULL rows give 0 (the Nullable(UInt8) result folded for filters)
            ColumnPtr a = materialize(ctx_, block.getByName(act.a).column);
            auto c = std::const_pointer_cast<IColumn>(newColumn(ctx_, rt, n));
            if (n)
                check(tfg_cmp_const(ctx_.raw(), a->type.type, a->dataPtr(), a->nullPtr(), (int64_t)n, act.op,
                                    act.constant.type, &act.constant.bits, (uint8_t *)c->data->data()),
                      "tfg_cmp_const");
            res = c;
            break;
        }
        case 1: {
            ColumnPtr a = materialize(ctx_, block.getByName(act.a).column);
            ColumnPtr b = materialize(ctx_, block.getByName(act.b).column);
            auto c = std::const_pointer_cast<IColumn>(newColumn(ctx_, rt, n));
            if (n)
                check(tfg_cmp_vector(ctx_.raw(), a->type.type, a->dataPtr(), a->nullPtr(), act.op, b->type.type,
                                     b->dataPtr(), b->nullPtr(), (int64_t)n, (uint8_t *)c->data->data()),
                      "tfg_cmp_vector");
            res = c;
            break;
        }
        case 2: {
            ColumnPtr a = materialize(ctx_, block.getByName(act.a).column);
            ColumnPtr b = act.op == TFG_NOT ? a : materialize(ctx_, block.getByName(act.b).column);
            auto c = std::const_pointer_cast<IColumn>(newColumn(ctx_, rt, n));
            if (n)
                check(tfg_mask_logic(ctx_.raw(), act.op, (const uint8_t *)a->dataPtr(), (const uint8_t *)b->dataPtr(),
                                     (int64_t)n, (uint8_t *)c->data->data()),
                      "tfg_mask_logic");
            res = c;
            break;
        }
        case 5: { // constant Op column (e.g. 1 - l_discount): the constant-vector form of tfg_arith
            ColumnPtr b = materialize(ctx_, block.getByName(act.b).column);
            DataType at;
            at.type = act.constant.type;
            at.scale = act.constant.scale;
            at.prec = act.constant.prec;
            rt = arithResult(act.op, at, b->type);
            auto c = std::const_pointer_cast<IColumn>(newColumn(ctx_, rt, n));
            if (n)
                check(tfg_arith(ctx_.raw(), act.op, at.type, &act.constant.bits, 1, at.scale, b->type.type, b->dataPtr(), 0,
                                b->type.scale, rt.type, rt.scale, (int64_t)n, c->data->data()),
                      "tfg_arith");
            c->nullmap = mergeNulls(ctx_, *b, nullptr, n);
            c->type.nullable = c->nullmap != nullptr;
            rt.nullable = c->type.nullable;
            res = c;
            break;
        }
        default: { // arithmetic, column or constant right operand
            ColumnPtr a = materialize(ctx_, block.getByName(act.a).column);
            ColumnPtr b;
            DataType bt;
            const void *bp;
            int b_const = 0;
            if (act.kind == 3) {
                b = materialize(ctx_, block.getByName(act.b).column);
                bt = b->type;
                bp = b->dataPtr();
            } else {
                bt.type = act.constant.type;
                bt.scale = act.constant.scale;
                bt.prec = act.constant.prec;
                bp = &act.constant.bits;
                b_const = 1;
            }
            rt = arithResult(act.op, a->type, bt);
            auto c = std::const_pointer_cast<IColumn>(newColumn(ctx_, rt, n));
            if (n)
                check(tfg_arith(ctx_.raw(), act.op, a->type.type, a->dataPtr(), 0, a->type.scale, bt.type, bp, b_const,
                                bt.scale, rt.type, rt.scale, (int64_t)n, c->data->data()),
                      "tfg_arith");
            c->nullmap = mergeNulls(ctx_, *a, b.get(), n);
            c->type.nullable = c->nullmap != nullptr;
            rt.nullable = c->type.nullable;
            res = c;
            break;
        }
        }
        block.insert({res, res->type, act.result});
    }
}

// ---------------------------------------------------------------- FilterTransformAction
FilterTransformAction::FilterTransformAction(Context &ctx, const Block &header, ExpressionActionsPtr expression,
                                             const std::string &filter_column_name)
    : ctx_(ctx), header_(header.cloneEmpty()), expression_(std::move(expression)), filter_column_name_(filter_column_name) {
    if (!header_.has(filter_column_name_)) {
        DataType t;
        t.type = TFG_UINT8;
        header_.insert({nullptr, t, filter_column_name_});
    }
}

bool FilterTransformAction::transform(Block &block, FilterPtr &res_filter, bool return_filter) {
    if (!block) return true;
    if (expression_) expression_->execute(block);
    const size_t pos = block.getPositionByName(filter_column_name_);
    const size_t rows = block.rows();
    ColumnPtr column_of_filter = block.safeGetByPosition(pos).column;
    DataType u8;
    u8.type = TFG_UINT8;
    if (column_of_filter->is_const) { // ConstantFilterDescription
        if (column_of_filter->const_value == 0) {
            block.clear();
            return true;
        }
        if (return_filter) res_filter = nullptr;
        return true;
    }
    if (column_of_filter->type.type != TFG_UINT8 && column_of_filter->type.type != TFG_INT8)
        throw Exception("Illegal type " + column_of_filter->type.getName() + " of column for filter",
                        ErrorCodes::ILLEGAL_TYPE_OF_COLUMN_FOR_FILTER);
    // FilterDescription: Nullable(UInt8) -> v && !null
    ColumnPtr filter = column_of_filter;
    if (column_of_filter->nullmap) {
        auto f = std::make_shared<IColumn>();
        f->type = u8;
        f->rows = rows;
        f->data = std::make_shared<DeviceBuffer>(ctx_, rows);
        DeviceBuffer notnull(ctx_, rows);
        check(tfg_mask_logic(ctx_.raw(), TFG_NOT, column_of_filter->nullPtr(), nullptr, (int64_t)rows,
                             (uint8_t *)notnull.data()),
              "tfg_mask_logic");
        check(tfg_mask_logic(ctx_.raw(), TFG_AND, (const uint8_t *)column_of_filter->dataPtr(),
                             (const uint8_t *)notnull.data(), (int64_t)rows, (uint8_t *)f->data->data()),
              "tfg_mask_logic");
        ctx_.sync();
        filter = f;
    }
    if (return_filter) {
        res_filter = filter;
        return true;
    }
    uint64_t filtered_rows = 0;
    check(tfg_count_mask(ctx_.raw(), (const uint8_t *)filter->dataPtr(), nullptr, (int64_t)rows, nullptr, &filtered_rows),
          "tfg_count_mask");
    if (filtered_rows == 0) return false;
    if (filtered_rows == rows) {
        auto &fc = block.safeGetByPosition(pos);
        fc.column = makeConstColumn(fc.type, 1, filtered_rows);
        return true;
    }
    // every fixed-width column (and null map) of the block in one compaction launch
    std::vector<const void *> ins;
    std::vector<void *> outs;
    std::vector<int> widths;
    std::vector<ColumnPtr> results(block.columns());
    for (size_t i = 0; i < block.columns(); ++i) {
        const ColumnWithTypeAndName &cur = block.safeGetByPosition(i);
        const IColumn &c = *cur.column;
        if (i == pos) {
            results[i] = makeConstColumn(cur.type, 1, filtered_rows);
            continue;
        }
        if (c.is_const) {
            results[i] = makeConstColumn(c.type, c.const_value, filtered_rows);
            continue;
        }
        auto r = std::make_shared<IColumn>();
        r->type = c.type;
        r->rows = filtered_rows;
        if (c.type.isString()) {
            r->offsets = std::make_shared<DeviceBuffer>(ctx_, filtered_rows * 8);
            r->data = std::make_shared<DeviceBuffer>(ctx_, c.chars); // upper bound
            uint64_t out_rows = 0, out_bytes = 0;
            check(tfg_filter_string(ctx_.raw(), (const uint8_t *)filter->dataPtr(), (int64_t)rows,
                                    (const uint8_t *)c.dataPtr(), (const uint64_t *)c.offsets->data(),
                                    (uint8_t *)r->data->data(), (uint64_t *)r->offsets->data(), &out_rows, &out_bytes),
                  "tfg_filter_string");
            r->chars = out_bytes;
        } else {
            r->data = std::make_shared<DeviceBuffer>(ctx_, filtered_rows * c.type.width());
            ins.push_back(c.dataPtr());
            outs.push_back(r->data->data());
            widths.push_back((int)c.type.width());
        }
        if (c.nullmap) {
            r->nullmap = std::make_shared<DeviceBuffer>(ctx_, filtered_rows);
            ins.push_back(c.nullPtr());
            outs.push_back(r->nullmap->data());
            widths.push_back(1);
        }
        results[i] = r;
    }
    if (!ins.empty()) {
        uint64_t cnt = 0;
        check(tfg_filter(ctx_.raw(), (const uint8_t *)filter->dataPtr(), (int64_t)rows, (int)ins.size(), ins.data(),
                         widths.data(), outs.data(), nullptr, &cnt),
              "tfg_filter");
        if (cnt != filtered_rows) throw Exception("filter count mismatch", ErrorCodes::LOGICAL_ERROR);
    }
    for (size_t i = 0; i < block.columns(); ++i) block.safeGetByPosition(i).column = results[i];
    return true;
}

// ---------------------------------------------------------------- FilterBlockInputStream
FilterBlockInputStream::FilterBlockInputStream(Context &ctx, BlockInputStreamPtr input, ExpressionActionsPtr expression,
                                               const std::string &filter_column)
    : input_(std::move(input)), action_(ctx, input_->getHeader(), std::move(expression), filter_column) {}

Block FilterBlockInputStream::read() {
    FilterPtr unused;
    for (;;) {
        Block b = input_->read();
        if (!b) return b;
        if (!action_.transform(b, unused, false)) continue; // every row filtered out
        if (!b) continue;                                     // constant false
        return b;
    }
}

} // namespace tfa
