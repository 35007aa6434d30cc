// operators.cpp — Aggregator, Join, HashPartitionWriter, MPPExchange and the block streams of the
// host layer, each a thin C++ facade over the C-ABI (tfa_host.h lists the reference interfaces).
#include <algorithm>
#include <cstring>

#include "tfa_host.h"

namespace tfa {

// ================================================================ Aggregator
Aggregator::Aggregator(Context &ctx, const Params &params) : ctx_(ctx), params_(params) {
    // chooseAggregationMethod (Aggregator.cpp:394-537): one fixed key -> key8..key64; several
    // fixed keys or one String key -> the packed 16-byte methods (keys128 / key_string), and
    // past those (String with other keys, wider tuples) serialized: tfg_agg_create_keys decides
    int key_type = 0;
    std::vector<int> packed_types;
    for (const auto &k : params_.keys) {
        key_types_.push_back(params_.src_header.getByName(k).type);
        packed_types.push_back(key_types_.back().isString() ? (int)TFG_STRING : key_types_.back().type);
    }
    if (!params_.keys.empty()) {
        key_type_ = key_types_[0];
        key_type = key_type_.type;
    }
    packed_ = params_.keys.size() > 1 || (!params_.keys.empty() && (key_type_.isString() || key_type_.width() > 8));
    std::vector<int> arg_types, arg_scales;
    for (const auto &d : params_.aggregates) {
        int kind;
        DataType at;
        int ref = -1;
        if (d.function == "first_row" && d.argument_names.size() == 1)
            for (size_t j = 0; j < params_.keys.size(); ++j)
                if (params_.keys[j] == d.argument_names[0]) ref = (int)j;
        ref_key_.push_back(ref);
        if (ref >= 0) { // first_row of a key: the key column itself, nothing on the device
            dev_index_.push_back(-1);
            continue;
        }
        dev_index_.push_back((int)kinds_.size());
        if (d.function == "min" || d.function == "max" || d.function == "first_row") {
            if (d.argument_names.size() != 1)
                throw Exception(d.function + " takes one argument", ErrorCodes::BAD_ARGUMENTS);
            kind = d.function == "min" ? TFG_AGG_MIN : d.function == "max" ? TFG_AGG_MAX : TFG_AGG_FIRST_ROW;
            at = params_.src_header.getByName(d.argument_names[0]).type;
        } else if (d.function == "sum") {
            if (d.argument_names.size() != 1)
                throw Exception("sum takes one argument", ErrorCodes::BAD_ARGUMENTS);
            kind = TFG_AGG_SUM;
            at = params_.src_header.getByName(d.argument_names[0]).type;
        } else if (d.function == "count") {
            if (d.argument_names.empty()) {
                kind = TFG_AGG_COUNT_ALL;
            } else {
                kind = TFG_AGG_COUNT;
                at = params_.src_header.getByName(d.argument_names[0]).type;
            }
        } else {
            throw Exception("Unknown aggregate function " + d.function, ErrorCodes::NOT_IMPLEMENTED);
        }
        if (at.isString() && kind != TFG_AGG_MIN && kind != TFG_AGG_MAX && kind != TFG_AGG_FIRST_ROW &&
            kind != TFG_AGG_COUNT)
            throw Exception(d.function + " over a String column", ErrorCodes::ILLEGAL_TYPE_OF_ARGUMENT);
        kinds_.push_back(kind);
        arg_types_.push_back(at);
        const int dev_type = at.isString() ? (int)TFG_STRING : at.type;
        arg_types.push_back(kind == TFG_AGG_COUNT_ALL
                                ? 0
                                : (dev_type | (at.nullable ? TFG_ARG_NULLABLE : 0) |
                                   (at.isDecimal() ? TFG_ARG_PREC(at.precision()) : 0) |
                                   (at.isString() && kind != TFG_AGG_COUNT ? TFG_ARG_COLLATOR(d.collator) : 0)));
        arg_scales.push_back(at.scale);
    }
    if (kinds_.empty()) { // only key references: the device aggregator still needs one aggregate
        hidden_count_ = true;
        kinds_.push_back(TFG_AGG_COUNT_ALL);
        arg_types_.push_back(DataType{});
        arg_types.push_back(0);
        arg_scales.push_back(0);
    }
    tfg_agg_params p{params_.bucket_bits, params_.expected_groups};
    if (packed_) {
        std::vector<int> coll = params_.collators;
        coll.resize(params_.keys.size(), TFG_COLLATOR_NONE);
        check(tfg_agg_create_keys(ctx_.raw(), (int)packed_types.size(), packed_types.data(), coll.data(),
                                  (int)kinds_.size(), kinds_.data(), arg_types.data(), arg_scales.data(), &p, &agg_),
              "tfg_agg_create_keys");
        return;
    }
    check(tfg_agg_create(ctx_.raw(), key_type, (int)kinds_.size(), kinds_.data(), arg_types.data(), arg_scales.data(),
                         &p, &agg_),
          "tfg_agg_create");
}

void Aggregator::keyPointers(const Block &b, std::vector<const void *> &cols, std::vector<const uint64_t *> &offs,
                             std::vector<const uint8_t *> &nulls, std::vector<ColumnPtr> &hold) const {
    for (const auto &k : params_.keys) {
        ColumnPtr c = materialize(ctx_, b.getByName(k).column);
        hold.push_back(c);
        cols.push_back(c->dataPtr());
        offs.push_back(c->offsets ? (const uint64_t *)c->offsets->data() : nullptr);
        nulls.push_back(c->nullPtr());
    }
}

Aggregator::~Aggregator() {
    if (agg_) tfg_agg_destroy(agg_);
}

// the device argument of a column: its values, or (String) a tfg_str_col kept in `strs`
static const void *devArg(const ColumnPtr &c, std::vector<std::unique_ptr<tfg_str_col>> &strs) {
    if (!c->type.isString()) return c->dataPtr();
    strs.push_back(std::make_unique<tfg_str_col>(
        tfg_str_col{(const uint8_t *)c->dataPtr(), c->offsets ? (const uint64_t *)c->offsets->data() : nullptr}));
    return strs.back().get();
}

void Aggregator::argPointers(const Block &b, std::vector<const void *> &args, std::vector<const uint8_t *> &nulls,
                             std::vector<ColumnPtr> &hold, std::vector<std::unique_ptr<tfg_str_col>> &strs) const {
    for (size_t i = 0; i < params_.aggregates.size() + (hidden_count_ ? 1 : 0); ++i) {
        if (i < params_.aggregates.size() && dev_index_[i] < 0) continue; // a key reference
        const int k = hidden_count_ ? TFG_AGG_COUNT_ALL : kinds_[dev_index_[i]];
        if (k == TFG_AGG_COUNT_ALL) {
            args.push_back(nullptr);
            nulls.push_back(nullptr);
            continue;
        }
        ColumnPtr c = materialize(ctx_, b.getByName(params_.aggregates[i].argument_names[0]).column);
        hold.push_back(c);
        args.push_back(k == TFG_AGG_COUNT ? c->dataPtr() : devArg(c, strs)); // count reads the null map only
        nulls.push_back(c->nullPtr());
    }
}

void Aggregator::executeOnBlock(const Block &block, const FilterPtr &filter) {
    const size_t n = block.rows();
    std::vector<const void *> args;
    std::vector<const uint8_t *> nulls;
    std::vector<ColumnPtr> hold;
    std::vector<std::unique_ptr<tfg_str_col>> strs;
    argPointers(block, args, nulls, hold, strs);
    if (packed_) {
        std::vector<const void *> kc;
        std::vector<const uint64_t *> ko;
        std::vector<const uint8_t *> kn;
        keyPointers(block, kc, ko, kn, hold);
        check(tfg_agg_consume_keys(agg_, kc.data(), ko.data(), kn.data(), args.data(), nulls.data(),
                                   filter ? (const uint8_t *)filter->dataPtr() : nullptr, (int64_t)n),
              "tfg_agg_consume_keys");
        return;
    }
    ColumnPtr key;
    if (!params_.keys.empty()) key = materialize(ctx_, block.getByName(params_.keys[0]).column);
    check(tfg_agg_consume(agg_, key ? key->dataPtr() : nullptr, key ? key->nullPtr() : nullptr, args.data(), nulls.data(),
                          filter ? (const uint8_t *)filter->dataPtr() : nullptr, (int64_t)n),
          "tfg_agg_consume");
}

void Aggregator::executeOnBlockFiltered(const Block &block, const std::string &pred, int op, Field constant) {
    const size_t n = block.rows();
    if (packed_) { // the predicate's mask, then the packed-key consume
        ColumnPtr p = materialize(ctx_, block.getByName(pred).column);
        auto m = std::make_shared<IColumn>();
        m->type.type = TFG_UINT8;
        m->rows = n;
        m->data = std::make_shared<DeviceBuffer>(ctx_, std::max<size_t>(n, 1));
        if (n)
            check(tfg_cmp_const(ctx_.raw(), p->type.type, p->dataPtr(), p->nullPtr(), (int64_t)n, op, constant.type,
                                &constant.bits, (uint8_t *)m->data->data()),
                  "tfg_cmp_const");
        executeOnBlock(block, m);
        return;
    }
    std::vector<const void *> args;
    std::vector<const uint8_t *> nulls;
    std::vector<ColumnPtr> hold;
    std::vector<std::unique_ptr<tfg_str_col>> strs;
    argPointers(block, args, nulls, hold, strs);
    ColumnPtr key;
    if (!params_.keys.empty()) key = materialize(ctx_, block.getByName(params_.keys[0]).column);
    ColumnPtr p = materialize(ctx_, block.getByName(pred).column);
    check(tfg_agg_consume_filtered(agg_, p->type.type, p->dataPtr(), p->nullPtr(), op, constant.type, &constant.bits,
                                   key ? key->dataPtr() : nullptr, key ? key->nullPtr() : nullptr, args.data(),
                                   nulls.data(), (int64_t)n),
          "tfg_agg_consume_filtered");
}

void Aggregator::mergeOnBlock(const Block &partial) {
    const size_t n = partial.rows();
    std::vector<const void *> states;
    std::vector<const uint8_t *> nulls;
    std::vector<ColumnPtr> hold;
    std::vector<std::unique_ptr<tfg_str_col>> strs;
    for (size_t i = 0; i < params_.aggregates.size(); ++i) {
        if (dev_index_[i] < 0) continue; // a key reference: the keys carry it
        ColumnPtr c = materialize(ctx_, partial.getByName(params_.aggregates[i].column_name).column);
        hold.push_back(c);
        states.push_back(devArg(c, strs));
        nulls.push_back(c->nullPtr());
    }
    std::shared_ptr<DeviceBuffer> zeros;
    if (hidden_count_) { // partial counts of the hidden count(): never output, any value will do
        zeros = std::make_shared<DeviceBuffer>(ctx_, std::max<size_t>(n, 1) * 8);
        states.push_back(zeros->data());
        nulls.push_back(nullptr);
    }
    if (packed_) {
        std::vector<const void *> kc;
        std::vector<const uint64_t *> ko;
        std::vector<const uint8_t *> kn;
        keyPointers(partial, kc, ko, kn, hold);
        check(tfg_agg_consume_partial_keys(agg_, kc.data(), ko.data(), kn.data(), states.data(), nulls.data(),
                                           (int64_t)n),
              "tfg_agg_consume_partial_keys");
        return;
    }
    ColumnPtr key;
    if (!params_.keys.empty()) key = materialize(ctx_, partial.getByName(params_.keys[0]).column);
    check(tfg_agg_consume_partial(agg_, key ? key->dataPtr() : nullptr, key ? key->nullPtr() : nullptr, states.data(),
                                  nulls.data(), (int64_t)n),
          "tfg_agg_consume_partial");
}

void Aggregator::merge(Aggregator &other) { check(tfg_agg_merge(agg_, other.agg_), "tfg_agg_merge"); }

size_t Aggregator::size() const {
    uint64_t g = 0;
    check(tfg_agg_size(agg_, &g), "tfg_agg_size");
    return g;
}

void Aggregator::reset() { check(tfg_agg_reset(agg_), "tfg_agg_reset"); }

Block Aggregator::convertToBlock(bool final) const {
    (void)final; // partial and final blocks have the same layout: state = result value + NULL flag
    const size_t g = size();
    Block out;
    std::shared_ptr<IColumn> key;
    if (!params_.keys.empty() && !packed_) {
        key = std::make_shared<IColumn>();
        key->type = key_type_;
        key->rows = g;
        key->data = std::make_shared<DeviceBuffer>(ctx_, g * key_type_.width());
        if (key_type_.nullable) key->nullmap = std::make_shared<DeviceBuffer>(ctx_, g);
    }
    std::vector<std::shared_ptr<IColumn>> states;
    std::vector<void *> sp;
    std::vector<uint8_t *> snp;
    std::vector<std::unique_ptr<tfg_str_out>> souts; // String results (min / max / first_row of a String)
    for (size_t i = 0; i < kinds_.size(); ++i) { // the device aggregates
        int t = 0, w = 0;
        check(tfg_agg_result_type(agg_, (int)i, &t, &w), "tfg_agg_result_type");
        auto c = std::make_shared<IColumn>();
        const bool ord = kinds_[i] == TFG_AGG_MIN || kinds_[i] == TFG_AGG_MAX || kinds_[i] == TFG_AGG_FIRST_ROW;
        if (t == TFG_STRING) {
            uint64_t bytes = 0;
            check(tfg_agg_result_chars(agg_, (int)i, &bytes), "tfg_agg_result_chars");
            c->type.type = DataType::TYPE_STRING;
            c->type.nullable = arg_types_[i].nullable || kinds_[i] == TFG_AGG_FIRST_ROW;
            c->rows = g;
            c->chars = bytes;
            c->data = std::make_shared<DeviceBuffer>(ctx_, std::max<uint64_t>(bytes, 1));
            c->offsets = std::make_shared<DeviceBuffer>(ctx_, std::max<size_t>(g, 1) * 8);
            if (c->type.nullable) c->nullmap = std::make_shared<DeviceBuffer>(ctx_, std::max<size_t>(g, 1));
            souts.push_back(std::make_unique<tfg_str_out>(
                tfg_str_out{(uint8_t *)c->data->data(), (uint64_t *)c->offsets->data(), bytes}));
            sp.push_back(souts.back().get());
            snp.push_back(c->nullmap ? (uint8_t *)c->nullmap->data() : nullptr);
            states.push_back(c);
            continue;
        }
        c->type.type = t;
        c->type.scale = kinds_[i] == TFG_AGG_SUM || ord ? arg_types_[i].scale : 0;
        if (ord) c->type.prec = arg_types_[i].prec; // min / max / first_row: the argument's type
        // sum(Decimal(p, s)) -> Decimal(min(p + 22, 65), s) (SumDecimalInferer, Common/Decimal.h:156-163)
        if (kinds_[i] == TFG_AGG_SUM && arg_types_[i].isDecimal())
            c->type.prec = std::min(arg_types_[i].precision() + 22, 65);
        // sum / min / max over a nullable argument are Nullable (AggregateFunctionNullUnary);
        // first_row always is (AggregateFunctionFirstRowNull, the reference's first_row column
        // types: gtest_aggregation_executor.cpp:1129); count never is
        c->type.nullable = ((kinds_[i] == TFG_AGG_SUM || ord) && arg_types_[i].nullable) || kinds_[i] == TFG_AGG_FIRST_ROW;
        c->rows = g;
        c->data = std::make_shared<DeviceBuffer>(ctx_, g * (size_t)w);
        if (c->type.nullable) c->nullmap = std::make_shared<DeviceBuffer>(ctx_, g);
        sp.push_back(c->data->data());
        snp.push_back(c->nullmap ? (uint8_t *)c->nullmap->data() : nullptr);
        states.push_back(c);
    }
    uint64_t got = 0;
    if (packed_) { // convertToBlockImplFinal with the packed keys unpacked into their columns
        std::vector<std::shared_ptr<IColumn>> kcols;
        std::vector<void *> kp;
        std::vector<uint64_t *> ko;
        std::vector<uint8_t *> kn;
        for (const DataType &t : key_types_) {
            auto c = std::make_shared<IColumn>();
            c->type = t;
            c->rows = g;
            if (t.isString()) {
                c->offsets = std::make_shared<DeviceBuffer>(ctx_, std::max<size_t>(g, 1) * 8);
            } else {
                c->data = std::make_shared<DeviceBuffer>(ctx_, std::max<size_t>(g, 1) * t.width());
            }
            if (t.nullable) c->nullmap = std::make_shared<DeviceBuffer>(ctx_, std::max<size_t>(g, 1));
            kcols.push_back(c);
        }
        uint64_t chars = 0;
        bool has_str = false;
        for (const DataType &t : key_types_) has_str |= t.isString();
        if (has_str) { // chars size first (TFG_ERR_CAPACITY reports the largest String key's)
            DeviceBuffer probe(ctx_, 8);
            std::vector<void *> pk(kcols.size(), probe.data());
            std::vector<uint64_t *> po(kcols.size(), (uint64_t *)probe.data());
            const int rc = tfg_agg_result_keys(agg_, pk.data(), po.data(), nullptr, nullptr, nullptr, g, 0, &got, &chars);
            if (rc != TFG_ERR_CAPACITY) check(rc, "tfg_agg_result_keys");
            for (auto &c : kcols)
                if (c->type.isString()) c->data = std::make_shared<DeviceBuffer>(ctx_, std::max<uint64_t>(chars, 1));
        }
        for (auto &c : kcols) {
            kp.push_back(c->data->data());
            ko.push_back(c->offsets ? (uint64_t *)c->offsets->data() : nullptr);
            kn.push_back(c->nullmap ? (uint8_t *)c->nullmap->data() : nullptr);
        }
        check(tfg_agg_result_keys(agg_, kp.data(), ko.data(), kn.data(), sp.data(), snp.data(), g, chars, &got,
                                  &chars),
              "tfg_agg_result_keys");
        ctx_.sync();
        for (auto &c : kcols) // each String column's own chars: its last end offset
            if (c->type.isString()) {
                uint64_t end = 0;
                if (g) check(tfg_download(ctx_.raw(), &end, (const uint64_t *)c->offsets->data() + (g - 1), 8),
                             "tfg_download");
                c->chars = end;
            }
        for (size_t j = 0; j < kcols.size(); ++j) out.insert({kcols[j], kcols[j]->type, params_.keys[j]});
        insertAggregateColumns(out, states, std::vector<ColumnPtr>(kcols.begin(), kcols.end()), g);
        return out;
    }
    check(tfg_agg_result(agg_, key ? key->data->data() : nullptr, key && key->nullmap ? (uint8_t *)key->nullmap->data() : nullptr,
                         sp.data(), snp.data(), g, &got),
          "tfg_agg_result");
    ctx_.sync();
    if (key) out.insert({key, key->type, params_.keys[0]});
    insertAggregateColumns(out, states, key ? std::vector<ColumnPtr>{key} : std::vector<ColumnPtr>{}, g);
    return out;
}

// aggregate columns in their declared order: a device aggregate's result, or (first_row of a
// GROUP BY column) the key column itself, Nullable like every first_row result
void Aggregator::insertAggregateColumns(Block &out, const std::vector<std::shared_ptr<IColumn>> &states,
                                        const std::vector<ColumnPtr> &keys, size_t g) const {
    for (size_t i = 0; i < params_.aggregates.size(); ++i) {
        const std::string &name = params_.aggregates[i].column_name;
        if (dev_index_[i] >= 0) {
            out.insert({states[dev_index_[i]], states[dev_index_[i]]->type, name});
            continue;
        }
        ColumnPtr k = keys.at(ref_key_[i]);
        if (k->type.nullable) {
            out.insert({k, k->type, name});
            continue;
        }
        auto c = std::make_shared<IColumn>(*k); // shares the key's buffers
        c->type.nullable = true;
        c->nullmap = std::make_shared<DeviceBuffer>(ctx_, std::max<size_t>(g, 1));
        check(tfg_memset(ctx_.raw(), c->nullmap->data(), 0, std::max<size_t>(g, 1)), "tfg_memset");
        out.insert({c, c->type, name});
    }
}

// ================================================================ Join
Join::Join(Context &ctx, JoinKind kind, const std::string &probe_key, const std::string &build_key,
           int64_t expected_build_rows)
    : Join(ctx, kind, std::vector<std::string>{probe_key}, std::vector<std::string>{build_key}, expected_build_rows) {}

Join::Join(Context &ctx, JoinKind kind, std::vector<std::string> probe_keys, std::vector<std::string> build_keys,
           int64_t expected_build_rows, std::vector<int> collators)
    : ctx_(ctx), kind_(kind), probe_keys_(std::move(probe_keys)), build_keys_(std::move(build_keys)),
      collators_(std::move(collators)), expected_(expected_build_rows) {
    if (probe_keys_.empty() || probe_keys_.size() != build_keys_.size())
        throw Exception("join needs the same number (>= 1) of probe and build keys", ErrorCodes::BAD_ARGUMENTS);
    collators_.resize(build_keys_.size(), TFG_COLLATOR_NONE);
}

Join::~Join() {
    if (join_) tfg_join_destroy(join_);
}

void Join::initBuild(const Block &sample_block) {
    sample_ = sample_block.cloneEmpty();
    // chooseJoinMapMethod (JoinHashMap.cpp:33-116): one integer key of <= 8 bytes joins on its
    // value (key8..key64); anything else on the key tuple's fingerprint, verified per pair
    const DataType kt = sample_.getByName(build_keys_[0]).type;
    general_keys_ = build_keys_.size() > 1 || kt.isString() || kt.width() > 8 || kt.type == TFG_FLOAT32 ||
                    kt.type == TFG_FLOAT64;
    if (v2_flags_ >= 0)
        check(tfg_join_create_v2(ctx_.raw(), general_keys_ ? (int)TFG_UINT64 : kt.type, expected_, v2_flags_, &join_),
              "tfg_join_create_v2");
    else
        check(tfg_join_create(ctx_.raw(), general_keys_ ? (int)TFG_UINT64 : kt.type, expected_, &join_),
              "tfg_join_create");
}

// The column the table is keyed on: the key itself, or (general keys) the UInt64 fingerprint
// of the tuple with the OR of the key null maps.
ColumnPtr Join::joinKey(const Block &block, const std::vector<std::string> &names) const {
    if (!general_keys_) return materialize(ctx_, block.getByName(names[0]).column);
    const size_t n = block.rows(), nk = names.size();
    std::vector<ColumnPtr> hold(nk);
    std::vector<int> types(nk);
    std::vector<const void *> cols(nk);
    std::vector<const uint64_t *> offs(nk);
    std::vector<const uint8_t *> nulls(nk);
    for (size_t j = 0; j < nk; ++j) {
        hold[j] = materialize(ctx_, block.getByName(names[j]).column);
        types[j] = hold[j]->type.isString() ? (int)TFG_STRING : hold[j]->type.type;
        cols[j] = hold[j]->dataPtr();
        offs[j] = hold[j]->offsets ? (const uint64_t *)hold[j]->offsets->data() : nullptr;
        nulls[j] = hold[j]->nullPtr();
    }
    auto c = std::make_shared<IColumn>();
    c->type.type = TFG_UINT64;
    c->type.nullable = true;
    c->rows = n;
    c->data = std::make_shared<DeviceBuffer>(ctx_, std::max<size_t>(n, 1) * 8);
    c->nullmap = std::make_shared<DeviceBuffer>(ctx_, std::max<size_t>(n, 1));
    check(tfg_join_key_hash(ctx_.raw(), (int)nk, types.data(), collators_.data(), cols.data(), offs.data(),
                            nulls.data(), (int64_t)n, (uint64_t *)c->data->data(), (uint8_t *)c->nullmap->data()),
          "tfg_join_key_hash");
    ctx_.sync();
    return c;
}

// pass[i] && the full key tuples of pair i are equal (general keys only)
DeviceBufferPtr Join::verifyKeys(const Block &probe_block, const uint32_t *pi, const uint32_t *bi, uint64_t count,
                                 DeviceBufferPtr pass) const {
    const size_t nk = probe_keys_.size();
    std::vector<ColumnPtr> hold;
    std::vector<int> types(nk);
    std::vector<const void *> pc(nk), bc(nk);
    std::vector<const uint64_t *> po(nk), bo(nk);
    for (size_t j = 0; j < nk; ++j) {
        ColumnPtr p = materialize(ctx_, probe_block.getByName(probe_keys_[j]).column);
        ColumnPtr b = materialize(ctx_, build_.getByName(build_keys_[j]).column);
        if (p->type.type != b->type.type)
            throw Exception("join key " + probe_keys_[j] + ": probe and build types differ",
                            ErrorCodes::ILLEGAL_TYPE_OF_ARGUMENT);
        types[j] = p->type.isString() ? (int)TFG_STRING : p->type.type;
        pc[j] = p->dataPtr();
        bc[j] = b->dataPtr();
        po[j] = p->offsets ? (const uint64_t *)p->offsets->data() : nullptr;
        bo[j] = b->offsets ? (const uint64_t *)b->offsets->data() : nullptr;
        hold.push_back(p);
        hold.push_back(b);
    }
    auto out = std::make_shared<DeviceBuffer>(ctx_, std::max<uint64_t>(count, 1));
    check(tfg_join_keys_equal(ctx_.raw(), (int)nk, types.data(), collators_.data(), pc.data(), po.data(), bc.data(),
                              bo.data(), pi, bi, pass ? (const uint8_t *)pass->data() : nullptr, (int64_t)count,
                              (uint8_t *)out->data()),
          "tfg_join_keys_equal");
    ctx_.sync();
    return out;
}

void Join::insertFromBlock(const Block &block) {
    if (!join_) initBuild(block);
    if (finished_) throw Exception("insertFromBlock after finishOneBuild", ErrorCodes::LOGICAL_ERROR);
    ColumnPtr k = joinKey(block, build_keys_);
    check(tfg_join_build(join_, k->dataPtr(), k->nullPtr(), (int64_t)block.rows()), "tfg_join_build");
    build_blocks_.push_back(block);
}

void Join::finishOneBuild() {
    if (!join_) throw Exception("finishOneBuild before initBuild", ErrorCodes::LOGICAL_ERROR);
    check(tfg_join_finalize(join_), "tfg_join_finalize");
    build_ = concatenateBlocks(ctx_, build_blocks_);
    build_blocks_.clear();
    finished_ = true;
}

uint64_t Join::buildRows() const {
    uint64_t rows = 0, parts = 0;
    if (join_) check(tfg_join_stats(join_, &rows, &parts), "tfg_join_stats");
    return rows;
}

void Join::setOtherCondition(ExpressionActionsPtr expr, std::string filter_column) {
    other_cond_ = std::move(expr);
    other_filter_ = std::move(filter_column);
}

// Rows of `block` where the device mask (UInt8, n rows) is set, in order (FilterTransformAction).
static Block filterByMask(Context &ctx, const Block &block, DeviceBufferPtr mask, size_t n) {
    static const std::string tmp = "__join_mark";
    Block b = block;
    DataType u8;
    u8.type = TFG_UINT8;
    auto m = std::make_shared<IColumn>();
    m->type = u8;
    m->rows = n;
    m->data = std::move(mask);
    b.insert({m, u8, tmp});
    FilterTransformAction f(ctx, b.cloneEmpty(), nullptr, tmp);
    FilterPtr none;
    if (!f.transform(b, none, false)) { // nothing qualifies: zero-row columns of the same types
        Block e;
        for (const auto &c : block.getColumnsWithTypeAndName()) {
            ColumnPtr g = gatherColumn(ctx, *c.column, nullptr, 0, false);
            e.insert({g, g->type, c.name});
        }
        return e;
    }
    b.erase(b.getPositionByName(tmp));
    return b;
}

// Join::handleOtherConditions (Interpreters/Join.cpp:798-1150), restated over device pairs: INNER
// probe -> joined pairs -> condition (NULL = false) -> per probe row "some pair passed" flags
// (tfg_join_mark) -> the kind's result.  Output order: passing pairs, then (LEFT) the unmatched
// probe rows; compare unordered, as the reference's join tests do.
Block Join::joinBlockWithCondition(const Block &probe_block) {
    const size_t n = probe_block.rows();
    ColumnPtr k = joinKey(probe_block, probe_keys_);
    uint64_t cap = std::max<uint64_t>(n, 1), count = 0;
    DeviceBufferPtr pi, bi;
    for (;;) {
        pi = std::make_shared<DeviceBuffer>(ctx_, cap * 4);
        bi = std::make_shared<DeviceBuffer>(ctx_, cap * 4);
        const int rc = tfg_join_probe(join_, TFG_JOIN_INNER, k->dataPtr(), k->nullPtr(), (int64_t)n,
                                      (uint32_t *)pi->data(), (uint32_t *)bi->data(), cap, nullptr, &count);
        if (rc == TFG_ERR_CAPACITY) {
            cap = count;
            continue;
        }
        check(rc, "tfg_join_probe");
        break;
    }
    // pairs joined, condition evaluated -> pass mask over the pairs (null = all pass)
    DeviceBufferPtr pass;
    Block joined;
    for (const auto &c : probe_block.getColumnsWithTypeAndName()) {
        ColumnPtr g = gatherColumn(ctx_, *c.column, (const uint32_t *)pi->data(), count, false);
        joined.insert({g, g->type, c.name});
    }
    for (const auto &c : build_.getColumnsWithTypeAndName()) {
        if (joined.has(c.name)) continue;
        ColumnPtr g = gatherColumn(ctx_, *c.column, (const uint32_t *)bi->data(), count, false);
        joined.insert({g, g->type, c.name});
    }
    if (other_cond_ && count) {
        FilterTransformAction f(ctx_, joined.cloneEmpty(), other_cond_, other_filter_);
        Block tmp = joined;
        FilterPtr mask;
        f.transform(tmp, mask, /*return_filter=*/true); // Nullable(UInt8) folded: v && !null
        if (!tmp) { // constant false: no pair passes
            pass = std::make_shared<DeviceBuffer>(ctx_, count);
            check(tfg_memset(ctx_.raw(), pass->data(), 0, count), "tfg_memset");
        } else if (mask) {
            pass = mask->data;
        }
    }
    if (general_keys_ && count) // candidate pairs of equal fingerprints -> key-equal pairs
        pass = verifyKeys(probe_block, (const uint32_t *)pi->data(), (const uint32_t *)bi->data(), count, pass);
    if (kind_ == JoinKind::Inner) {
        if (!pass) return joined;
        return filterByMask(ctx_, joined, pass, count);
    }
    auto flags = std::make_shared<DeviceBuffer>(ctx_, std::max<size_t>(n, 1));
    check(tfg_memset(ctx_.raw(), flags->data(), 0, std::max<size_t>(n, 1)), "tfg_memset");
    check(tfg_join_mark(ctx_.raw(), (const uint32_t *)pi->data(), pass ? (const uint8_t *)pass->data() : nullptr,
                        (int64_t)count, (uint8_t *)flags->data()),
          "tfg_join_mark");
    auto notflags = std::make_shared<DeviceBuffer>(ctx_, std::max<size_t>(n, 1));
    if (n)
        check(tfg_mask_logic(ctx_.raw(), TFG_NOT, (const uint8_t *)flags->data(), nullptr, (int64_t)n,
                             (uint8_t *)notflags->data()),
              "tfg_mask_logic");
    ctx_.sync();
    switch (kind_) {
    case JoinKind::Semi: return filterByMask(ctx_, probe_block, flags, n);
    case JoinKind::Anti: return filterByMask(ctx_, probe_block, notflags, n);
    case JoinKind::LeftOuterSemi:
    case JoinKind::AntiLeftOuterSemi: {
        Block out = probe_block;
        DataType i8;
        i8.type = TFG_INT8;
        i8.nullable = true;
        auto m = std::make_shared<IColumn>();
        m->type = i8;
        m->rows = n;
        m->data = kind_ == JoinKind::LeftOuterSemi ? flags : notflags;
        m->nullmap = std::make_shared<DeviceBuffer>(ctx_, std::max<size_t>(n, 1));
        check(tfg_memset(ctx_.raw(), m->nullmap->data(), 0, std::max<size_t>(n, 1)), "tfg_memset");
        out.insert({m, i8, match_helper_});
        ctx_.sync();
        return out;
    }
    default: break;
    }
    // LEFT: passing pairs, then every probe row without one (build side NULL)
    uint64_t kept = count;
    DeviceBufferPtr pk = pi, bk = bi;
    if (pass) {
        pk = std::make_shared<DeviceBuffer>(ctx_, std::max<uint64_t>(count, 1) * 4);
        bk = std::make_shared<DeviceBuffer>(ctx_, std::max<uint64_t>(count, 1) * 4);
        const void *ins[2] = {pi->data(), bi->data()};
        void *outs[2] = {pk->data(), bk->data()};
        const int w[2] = {4, 4};
        check(tfg_filter(ctx_.raw(), (const uint8_t *)pass->data(), (int64_t)count, 2, ins, w, outs, nullptr, &kept),
              "tfg_filter");
    }
    std::vector<uint32_t> iota(std::max<size_t>(n, 1));
    for (size_t i = 0; i < n; ++i) iota[i] = (uint32_t)i;
    DeviceBuffer rows_dev(ctx_, iota.size() * 4);
    check(tfg_upload(ctx_.raw(), rows_dev.data(), iota.data(), iota.size() * 4), "tfg_upload");
    uint64_t unmatched = 0;
    const uint64_t total_cap = kept + n;
    auto pall = std::make_shared<DeviceBuffer>(ctx_, std::max<uint64_t>(total_cap, 1) * 4);
    auto ball = std::make_shared<DeviceBuffer>(ctx_, std::max<uint64_t>(total_cap, 1) * 4);
    if (kept) check(tfg_copy(ctx_.raw(), pall->data(), pk->data(), kept * 4), "tfg_copy");
    if (kept) check(tfg_copy(ctx_.raw(), ball->data(), bk->data(), kept * 4), "tfg_copy");
    {
        const void *ins[1] = {rows_dev.data()};
        void *outs[1] = {(uint8_t *)pall->data() + kept * 4};
        const int w[1] = {4};
        if (n)
            check(tfg_filter(ctx_.raw(), (const uint8_t *)notflags->data(), (int64_t)n, 1, ins, w, outs, nullptr,
                             &unmatched),
                  "tfg_filter");
    }
    std::vector<uint32_t> none(std::max<uint64_t>(unmatched, 1), 0xFFFFFFFFu);
    if (unmatched)
        check(tfg_upload(ctx_.raw(), (uint8_t *)ball->data() + kept * 4, none.data(), unmatched * 4), "tfg_upload");
    const uint64_t total = kept + unmatched;
    Block out;
    for (const auto &c : probe_block.getColumnsWithTypeAndName()) {
        ColumnPtr g = gatherColumn(ctx_, *c.column, (const uint32_t *)pall->data(), total, false);
        out.insert({g, g->type, c.name});
    }
    for (const auto &c : build_.getColumnsWithTypeAndName()) {
        if (out.has(c.name)) continue;
        ColumnPtr g = gatherColumn(ctx_, *c.column, (const uint32_t *)ball->data(), total, true);
        out.insert({g, g->type, c.name});
    }
    ctx_.sync();
    return out;
}

Block Join::joinBlock(const Block &probe_block) {
    if (!finished_) finishOneBuild();
    if (other_cond_ || general_keys_ || kind_ == JoinKind::LeftOuterSemi || kind_ == JoinKind::AntiLeftOuterSemi)
        return joinBlockWithCondition(probe_block);
    const size_t n = probe_block.rows();
    ColumnPtr k = joinKey(probe_block, probe_keys_);
    const bool pairs = kind_ == JoinKind::Inner || kind_ == JoinKind::Left;
    uint64_t cap = std::max<uint64_t>(n, 1), count = 0;
    std::shared_ptr<DeviceBuffer> pi, bi;
    for (;;) {
        pi = std::make_shared<DeviceBuffer>(ctx_, cap * 4);
        bi = pairs ? std::make_shared<DeviceBuffer>(ctx_, cap * 4) : nullptr;
        const int rc = tfg_join_probe(join_, (int)kind_, k->dataPtr(), k->nullPtr(), (int64_t)n, (uint32_t *)pi->data(),
                                      bi ? (uint32_t *)bi->data() : nullptr, cap, nullptr, &count);
        if (rc == TFG_ERR_CAPACITY) {
            cap = count;
            continue;
        }
        check(rc, "tfg_join_probe");
        break;
    }
    Block out;
    for (const auto &c : probe_block.getColumnsWithTypeAndName()) {
        ColumnPtr g = gatherColumn(ctx_, *c.column, (const uint32_t *)pi->data(), count, false);
        out.insert({g, g->type, c.name});
    }
    if (pairs) {
        for (const auto &c : build_.getColumnsWithTypeAndName()) {
            if (out.has(c.name)) continue; // same-named key columns appear once
            ColumnPtr g = gatherColumn(ctx_, *c.column, (const uint32_t *)bi->data(), count, kind_ == JoinKind::Left);
            out.insert({g, g->type, c.name});
        }
    }
    ctx_.sync();
    return out;
}

// ================================================================ partitioning / exchange
// Blocks with String columns or a selective row list: weak hash column by column (over the
// selective rows only, HashBaseWriterHelper.cpp:110-130), fillSelector, the stable partition
// permutation (IColumn::scatter's order), mapped back to block rows through the selective
// list, then every column gathered per partition (:176-200).
// fine_grained_stream_count S > 0: partition_num * S buckets, bucket = part * S + hash % S
// (fillSelectorForFineGrainedShuffle, HashBaseWriterHelper.cpp:64-84)
static std::vector<Block> hashPartitionBlockGather(Context &ctx, const Block &block, const std::vector<size_t> &key_ids,
                                                   uint32_t partition_num, const std::vector<int> &collators,
                                                   uint32_t fine_grained_stream_count = 0) {
    const uint32_t buckets = partition_num * std::max<uint32_t>(fine_grained_stream_count, 1);
    const BlockSelectivePtr &selp = block.info.selective;
    const uint64_t *sel = selp ? selp->data() : nullptr;
    const size_t n = selp ? selp->size() : block.rows();
    DeviceBuffer h(ctx, std::max<size_t>(n, 1) * 4), selector(ctx, std::max<size_t>(n, 1) * 4),
        perm(ctx, std::max<size_t>(n, 1) * 4), offs_dev(ctx, (buckets + 1) * 8);
    std::vector<uint64_t> offs(buckets + 1, 0);
    if (n) {
        check(tfg_weak_hash_init(ctx.raw(), (uint32_t *)h.data(), (int64_t)n), "tfg_weak_hash_init");
        for (size_t k = 0; k < key_ids.size(); ++k) {
            ColumnPtr c = materialize(ctx, block.safeGetByPosition(key_ids[k]).column);
            if (c->type.isString())
                check(tfg_weak_hash_update_string_selective(ctx.raw(), (const uint8_t *)c->dataPtr(),
                                                            (const uint64_t *)c->offsets->data(), c->nullPtr(), sel,
                                                            (int64_t)n,
                                                            k < collators.size() ? collators[k] : TFG_COLLATOR_NONE,
                                                            (uint32_t *)h.data()),
                      "tfg_weak_hash_update_string");
            else
                check(tfg_weak_hash_update_selective(ctx.raw(), c->type.type, c->dataPtr(), c->nullPtr(), sel,
                                                     (int64_t)n, (uint32_t *)h.data()),
                      "tfg_weak_hash_update");
        }
        check(tfg_fill_selector(ctx.raw(), (const uint32_t *)h.data(), (int64_t)n, partition_num,
                                fine_grained_stream_count, (uint32_t *)selector.data()),
              "tfg_fill_selector");
    }
    check(tfg_partition(ctx.raw(), (const uint32_t *)selector.data(), (int64_t)n, buckets,
                        (uint32_t *)perm.data(), (uint64_t *)offs_dev.data(), offs.data()),
          "tfg_partition");
    if (sel && n) // positions among the selective rows -> block rows
        check(tfg_selective_perm(ctx.raw(), sel, (const uint32_t *)perm.data(), (int64_t)n, (uint32_t *)perm.data()),
              "tfg_selective_perm");
    std::vector<Block> parts(buckets);
    for (uint32_t p = 0; p < buckets; ++p) {
        const uint32_t *pp = (const uint32_t *)perm.data() + offs[p];
        const size_t rows = offs[p + 1] - offs[p];
        for (const auto &c : block.getColumnsWithTypeAndName()) {
            ColumnPtr g = gatherColumn(ctx, *materialize(ctx, c.column), pp, rows, false);
            parts[p].insert({g, g->type, c.name});
        }
    }
    ctx.sync();
    return parts;
}

std::vector<Block> hashPartitionBlock(Context &ctx, const Block &block, const std::vector<size_t> &key_ids,
                                      uint32_t partition_num, const std::vector<int> &collators) {
    if (block.info.selective) return hashPartitionBlockGather(ctx, block, key_ids, partition_num, collators);
    for (const auto &c : block.getColumnsWithTypeAndName())
        if (c.type.isString()) return hashPartitionBlockGather(ctx, block, key_ids, partition_num, collators);
    const size_t n = block.rows();
    std::vector<int> types, key_idx(key_ids.begin(), key_ids.end());
    std::vector<const void *> cols;
    std::vector<const uint8_t *> nulls;
    std::vector<ColumnPtr> hold;
    // the null maps travel as extra UInt8 columns (never hashed)
    std::vector<int> null_col(block.columns(), -1);
    for (size_t j = 0; j < block.columns(); ++j) {
        ColumnPtr c = materialize(ctx, block.safeGetByPosition(j).column);
        if (c->type.isString()) throw Exception("partitioning String columns", ErrorCodes::NOT_IMPLEMENTED);
        hold.push_back(c);
        types.push_back(c->type.type);
        cols.push_back(c->dataPtr());
        nulls.push_back(c->nullPtr());
    }
    for (size_t j = 0; j < block.columns(); ++j) {
        if (!hold[j]->nullmap) continue;
        null_col[j] = (int)types.size();
        types.push_back(TFG_UINT8);
        cols.push_back(hold[j]->nullPtr());
        nulls.push_back(nullptr);
    }
    std::vector<DeviceBufferPtr> outs_buf;
    std::vector<void *> outs;
    for (size_t j = 0; j < types.size(); ++j) {
        outs_buf.push_back(std::make_shared<DeviceBuffer>(ctx, n * tfg_type_width(types[j])));
        outs.push_back(outs_buf.back()->data());
    }
    DeviceBuffer offs_dev(ctx, (partition_num + 1) * 8);
    std::vector<uint64_t> offs(partition_num + 1, 0);
    check(tfg_hash_partition(ctx.raw(), (int64_t)n, (int)key_idx.size(), key_idx.data(), (int)types.size(), types.data(),
                             cols.data(), nulls.data(), partition_num, outs.data(), (uint64_t *)offs_dev.data(), offs.data()),
          "tfg_hash_partition");
    std::vector<Block> parts(partition_num);
    for (uint32_t p = 0; p < partition_num; ++p) {
        const size_t r0 = offs[p], rows = offs[p + 1] - offs[p];
        for (size_t j = 0; j < block.columns(); ++j) {
            auto c = std::make_shared<IColumn>();
            c->type = hold[j]->type;
            c->rows = rows;
            const size_t w = c->type.width();
            c->data = std::make_shared<DeviceBuffer>(ctx, rows * w);
            check(tfg_copy(ctx.raw(), c->data->data(), (char *)outs[j] + r0 * w, rows * w), "tfg_copy");
            if (null_col[j] >= 0) {
                c->nullmap = std::make_shared<DeviceBuffer>(ctx, rows);
                check(tfg_copy(ctx.raw(), c->nullmap->data(), (char *)outs[null_col[j]] + r0, rows), "tfg_copy");
            }
            parts[p].insert({c, c->type, block.safeGetByPosition(j).name});
        }
    }
    ctx.sync();
    return parts;
}

HashPartitionWriter::HashPartitionWriter(Context &ctx, std::vector<size_t> partition_col_ids, uint32_t partition_num,
                                         Sink sink, int64_t batch_send_min_limit)
    : ctx_(ctx), partition_col_ids_(std::move(partition_col_ids)), partition_num_(partition_num), sink_(std::move(sink)),
      limit_(batch_send_min_limit < 0 ? (int64_t)8192 * partition_num : batch_send_min_limit) {
    if (partition_num_ == 0) throw Exception("partition_num must be positive", ErrorCodes::BAD_ARGUMENTS);
}

void HashPartitionWriter::write(const Block &block) {
    if (!block || block.rows() == 0) return;
    if (block.info.selective) { // only the listed rows travel (HashPartitionWriter.cpp:121-122, 159, 221)
        flush();
        if (block.info.selective->size() == 0) return;
        std::vector<Block> parts = hashPartitionBlock(ctx_, block, partition_col_ids_, partition_num_, collators_);
        for (uint32_t p = 0; p < partition_num_; ++p) sink_(p, std::move(parts[p]));
        return;
    }
    pending_.push_back(block);
    pending_rows_ += block.rows();
    if ((int64_t)pending_rows_ >= limit_) flush();
}

void HashPartitionWriter::flush() {
    if (pending_.empty()) return;
    Block all = concatenateBlocks(ctx_, pending_);
    pending_.clear();
    pending_rows_ = 0;
    std::vector<Block> parts = hashPartitionBlock(ctx_, all, partition_col_ids_, partition_num_, collators_);
    for (uint32_t p = 0; p < partition_num_; ++p) sink_(p, std::move(parts[p]));
}

std::vector<Block> fineGrainedPartitionBlock(Context &ctx, const Block &block, const std::vector<size_t> &key_ids,
                                             uint32_t partition_num, uint32_t stream_count,
                                             const std::vector<int> &collators) {
    if (stream_count == 0 || stream_count > 1024)
        throw Exception("fine_grained_shuffle_stream_count must be in (0, 1024]", ErrorCodes::BAD_ARGUMENTS);
    return hashPartitionBlockGather(ctx, block, key_ids, partition_num, collators, stream_count);
}

// ================================================================ FineGrainedShuffleWriter
FineGrainedShuffleWriter::FineGrainedShuffleWriter(Context &ctx, std::vector<size_t> partition_col_ids,
                                                   uint32_t partition_num, uint32_t stream_count, uint64_t batch_size,
                                                   Sink sink, uint64_t max_buffered_bytes)
    : ctx_(ctx), partition_col_ids_(std::move(partition_col_ids)), partition_num_(partition_num),
      stream_count_(stream_count), max_buffered_rows_(batch_size * stream_count), max_buffered_bytes_(max_buffered_bytes),
      sink_(std::move(sink)) {
    if (partition_num_ == 0) throw Exception("partition_num must be positive", ErrorCodes::BAD_ARGUMENTS);
    if (stream_count_ == 0 || stream_count_ > 1024)
        throw Exception("fine_grained_shuffle_stream_count must be in (0, 1024]", ErrorCodes::BAD_ARGUMENTS);
}

// FineGrainedShuffleWriter::write (FineGrainedShuffleWriter.cpp:117-141): rows are buffered; a
// flush follows when the buffer reaches batch_size * stream_count rows or max_buffered_bytes, or
// holds stream_count blocks
void FineGrainedShuffleWriter::write(const Block &block) {
    if (!header_set_ && block) {
        header_ = block.cloneEmpty();
        header_set_ = true;
    }
    const size_t rows = block.info.selective ? block.info.selective->size() : block.rows();
    if (rows > 0) {
        buffered_rows_ += rows;
        for (const auto &c : block.getColumnsWithTypeAndName()) {
            ColumnPtr m = c.column;
            buffered_bytes_ += (m->data ? m->data->bytes() : 0) + (m->offsets ? m->offsets->bytes() : 0) +
                               (m->nullmap ? m->nullmap->bytes() : 0);
        }
        blocks_.push_back(block);
    }
    if (buffered_rows_ >= max_buffered_rows_ || buffered_bytes_ >= max_buffered_bytes_ || blocks_.size() == stream_count_)
        flush();
}

// batchWriteFineGrainedShuffle (:159-228): every buffered block scattered into partition_num *
// stream_count buckets (weak hash of the partition columns -> fine-grained selector), then one
// packet per partition holding the non-empty buckets of its streams as V1 chunks with their
// stream ids (MPPTunnelSetHelper::ToFineGrainedPacket)
void FineGrainedShuffleWriter::flush() {
    if (buffered_rows_ == 0) return;
    const uint32_t nb = partition_num_ * stream_count_;
    std::vector<std::vector<Block>> pieces(nb);
    for (const Block &b : blocks_) {
        std::vector<Block> parts = hashPartitionBlockGather(ctx_, b, partition_col_ids_, partition_num_, collators_, stream_count_);
        for (uint32_t k = 0; k < nb; ++k)
            if (parts[k].rows()) pieces[k].push_back(std::move(parts[k]));
    }
    blocks_.clear();
    buffered_rows_ = buffered_bytes_ = 0;
    for (uint32_t p = 0; p < partition_num_; ++p) {
        FineGrainedPacket packet;
        for (uint32_t s = 0; s < stream_count_; ++s) {
            const std::vector<Block> &v = pieces[p * stream_count_ + s];
            if (v.empty()) continue; // empty chunks are not sent
            CHBlockChunkCodecV1 codec(ctx_, header_);
            DevicePacket chunk = codec.encode(v);
            if (chunk.empty()) continue;
            packet.chunks.push_back(std::move(chunk));
            packet.stream_ids.push_back(s);
        }
        sink_(p, std::move(packet));
    }
}

RcclTransport::RcclTransport(Context &ctx, int nranks, int rank, const uint8_t *unique_id, size_t id_len)
    : nranks_(nranks), rank_(rank) {
    check(tfg_comm_init(ctx.raw(), nranks, rank, unique_id, id_len, &comm_), "tfg_comm_init");
}

RcclTransport::~RcclTransport() {
    if (comm_) tfg_comm_destroy(comm_);
}

void RcclTransport::alltoallCountsN(int k, const uint64_t *send, uint64_t *recv) {
    check(tfg_alltoall_counts_n(comm_, k, send, recv), "tfg_alltoall_counts_n");
}

void RcclTransport::exchangeSlices(const std::vector<tfg_slice> &send, const std::vector<tfg_slice> &recv) {
    check(tfg_exchange_slices(comm_, (int)send.size(), send.data(), (int)recv.size(), recv.data()), "tfg_exchange_slices");
}

MPPExchange::MPPExchange(Context &ctx, int nranks, int rank, const uint8_t *unique_id, size_t id_len)
    : MPPExchange(ctx, std::make_shared<RcclTransport>(ctx, nranks, rank, unique_id, id_len)) {}

MPPExchange::MPPExchange(Context &ctx, std::shared_ptr<ExchangeTransport> transport)
    : ctx_(ctx), t_(std::move(transport)), nranks_(t_->nranks()), rank_(t_->rank()) {}

static Block emptyOfHeader(Context &ctx, const Block &header) { // zero-row columns of the header's types
    Block empty;
    for (const auto &c : header.getColumnsWithTypeAndName()) {
        auto z = std::make_shared<IColumn>();
        z->type = c.type;
        z->data = std::make_shared<DeviceBuffer>(ctx, 1);
        if (c.type.isString()) z->offsets = std::make_shared<DeviceBuffer>(ctx, 8);
        if (c.type.nullable) z->nullmap = std::make_shared<DeviceBuffer>(ctx, 1);
        empty.insert({z, z->type, c.name});
    }
    return empty;
}

// Zero-copy exchange.  Planes per column: a fixed-width column's values; a String column's end
// offsets (8 bytes a row, relative to its partition's chars, rebased on arrival) and its chars
// (bytes); a Nullable column's null map.  One counts exchange carries, per rank pair, the rows,
// every String column's chars bytes and every null plane's rows (0 when that partition has no
// null map: the receiver's null plane is zeroed first); then every (peer, plane) slice is sent
// from the partition block where it lies and received into the output column at its offset.
Block MPPExchange::exchange(const std::vector<Block> &partitions) {
    if ((int)partitions.size() != nranks_)
        throw Exception("exchange needs one block per rank", ErrorCodes::BAD_ARGUMENTS);
    const Block &proto = partitions[0];
    const size_t ncols = proto.columns();
    for (const Block &b : partitions)
        if (b.columns() != ncols) throw Exception("partitions of different schemas", ErrorCodes::LOGICAL_ERROR);
    // counts per rank pair: [0] rows, then one per String column (chars), then one per Nullable
    // column (null map rows, 0 = none)
    std::vector<int> str_of(ncols, -1), nul_of(ncols, -1);
    int K = 1;
    for (size_t j = 0; j < ncols; ++j)
        if (proto.safeGetByPosition(j).type.isString()) str_of[j] = K++;
    for (size_t j = 0; j < ncols; ++j)
        if (proto.safeGetByPosition(j).type.nullable) nul_of[j] = K++;
    const int P = nranks_;
    std::vector<ColumnPtr> cols((size_t)P * ncols);
    std::vector<uint64_t> send_cnt((size_t)P * K, 0), recv_cnt((size_t)P * K, 0);
    for (int p = 0; p < P; ++p) {
        const Block &b = partitions[p];
        send_cnt[(size_t)p * K] = b.rows();
        for (size_t j = 0; j < ncols; ++j) {
            if (!b.safeGetByPosition(j).column) { // a header-only block (cloneEmpty): sends nothing
                if (b.rows()) throw Exception("column without data in a non-empty block", ErrorCodes::LOGICAL_ERROR);
                continue;
            }
            ColumnPtr c = materialize(ctx_, b.safeGetByPosition(j).column);
            const DataType &t = proto.safeGetByPosition(j).type;
            if (c->type.isString() != t.isString() || c->rows != b.rows())
                throw Exception("partitions of different schemas", ErrorCodes::LOGICAL_ERROR);
            if (c->nullmap && !t.nullable) // it would be dropped
                throw Exception("null map on a column of non-Nullable type", ErrorCodes::LOGICAL_ERROR);
            if (str_of[j] >= 0) send_cnt[(size_t)p * K + str_of[j]] = c->chars;
            if (nul_of[j] >= 0) send_cnt[(size_t)p * K + nul_of[j]] = c->nullmap ? c->rows : 0;
            cols[(size_t)p * ncols + j] = c;
        }
    }
    t_->alltoallCountsN(K, send_cnt.data(), recv_cnt.data());
    // where each source's rows / chars land
    std::vector<uint64_t> row0(P + 1, 0);
    for (int p = 0; p < P; ++p) row0[p + 1] = row0[p] + recv_cnt[(size_t)p * K];
    const uint64_t total = row0[P];
    std::vector<std::vector<uint64_t>> chars0(K); // per String counter: the bytes before source p
    for (size_t j = 0; j < ncols; ++j)
        if (str_of[j] >= 0) {
            auto &c0 = chars0[str_of[j]];
            c0.assign(P + 1, 0);
            for (int p = 0; p < P; ++p) c0[p + 1] = c0[p] + recv_cnt[(size_t)p * K + str_of[j]];
        }
    Block out;
    std::vector<std::shared_ptr<IColumn>> outc(ncols);
    for (size_t j = 0; j < ncols; ++j) {
        const DataType t = proto.safeGetByPosition(j).type;
        auto c = std::make_shared<IColumn>();
        c->type = t;
        c->rows = total;
        if (t.isString()) {
            c->chars = chars0[str_of[j]][P];
            c->data = std::make_shared<DeviceBuffer>(ctx_, std::max<uint64_t>(c->chars, 1));
            c->offsets = std::make_shared<DeviceBuffer>(ctx_, std::max<uint64_t>(total, 1) * 8);
        } else {
            c->data = std::make_shared<DeviceBuffer>(ctx_, std::max<uint64_t>(total * t.width(), 1));
        }
        if (t.nullable) {
            c->nullmap = std::make_shared<DeviceBuffer>(ctx_, std::max<uint64_t>(total, 1));
            bool partial = false; // a source without a null map leaves its rows zero (not NULL)
            for (int p = 0; p < P; ++p) partial |= recv_cnt[(size_t)p * K + nul_of[j]] != recv_cnt[(size_t)p * K];
            if (partial && total) // a device memset, ordered before the slices that land on it
                check(tfg_memset(ctx_.raw(), c->nullmap->data(), 0, total), "tfg_memset");
        }
        outc[j] = c;
    }
    // the slices, peer by peer, in one plane order on both sides
    std::vector<tfg_slice> sends, recvs;
    for (int p = 0; p < P; ++p)
        for (size_t j = 0; j < ncols; ++j) {
            static const IColumn none{}; // a header-only block's column: no rows, no planes
            const IColumn &c = cols[(size_t)p * ncols + j] ? *cols[(size_t)p * ncols + j] : none;
            const DataType &t = proto.safeGetByPosition(j).type;
            IColumn &o = *outc[j];
            const uint64_t r = recv_cnt[(size_t)p * K];
            if (t.isString()) {
                sends.push_back({p, c.offsets ? c.offsets->data() : nullptr, c.rows * 8});
                recvs.push_back({p, (uint64_t *)o.offsets->data() + row0[p], r * 8});
                sends.push_back({p, c.data ? c.data->data() : nullptr, c.chars});
                recvs.push_back({p, (uint8_t *)o.data->data() + chars0[str_of[j]][p],
                                 recv_cnt[(size_t)p * K + str_of[j]]});
            } else {
                sends.push_back({p, c.data ? c.data->data() : nullptr, c.rows * t.width()});
                recvs.push_back({p, (uint8_t *)o.data->data() + row0[p] * t.width(), r * t.width()});
            }
            if (t.nullable) {
                sends.push_back({p, c.nullmap ? c.nullmap->data() : nullptr, c.nullmap ? c.rows : 0});
                recvs.push_back({p, (uint8_t *)o.nullmap->data() + row0[p], recv_cnt[(size_t)p * K + nul_of[j]]});
            }
        }
    t_->exchangeSlices(sends, recvs);
    for (size_t j = 0; j < ncols; ++j) // String end offsets: each source's relative to its own chars
        if (str_of[j] >= 0 && total)
            check(tfg_string_rebase_offsets(ctx_.raw(), (uint64_t *)outc[j]->offsets->data(), P, row0.data(),
                                            chars0[str_of[j]].data()),
                  "tfg_string_rebase_offsets");
    ctx_.sync(); // the partitions may be released on return
    for (size_t j = 0; j < ncols; ++j) out.insert({outc[j], outc[j]->type, proto.safeGetByPosition(j).name});
    return out;
}

// ================================================================ streams
AggregatingBlockInputStream::AggregatingBlockInputStream(Context &ctx, BlockInputStreamPtr input,
                                                         const Aggregator::Params &params, bool final)
    : ctx_(ctx), input_(std::move(input)), aggregator_(ctx, params), final_(final) {}

Block AggregatingBlockInputStream::getHeader() const { // the result block's structure
    if (!header_) header_ = aggregator_.convertToBlock(final_).cloneEmpty();
    return header_;
}

Block AggregatingBlockInputStream::read() {
    if (done_) return Block();
    done_ = true;
    while (Block b = input_->read()) aggregator_.executeOnBlock(b);
    return aggregator_.convertToBlock(final_);
}

Block HashJoinProbeBlockInputStream::read() {
    for (;;) {
        Block b = input_->read();
        if (!b) return b;
        Block out = join_->joinBlock(b);
        if (out.rows() > 0) return out;
    }
}

} // namespace tfa
