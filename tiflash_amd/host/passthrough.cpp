// passthrough.cpp — AutoPassThroughHashAggContext over the device aggregator (§8 f4).
// Reference: Operators/AutoPassThroughHashAggContext.cpp:24-243 (state machine),
// Operators/AutoPassThroughHashAggHelper.cpp (pass-through columns),
// Interpreters/Aggregator.cpp:1132-1160 (executeOnBlockCollectHitRate / executeOnBlockOnlyLookup).
#include "tfa_host.h"

namespace tfa {

AutoPassThroughHashAggContext::AutoPassThroughHashAggContext(Context &ctx, const Aggregator::Params &params,
                                                             uint64_t row_limit_unit, uint64_t normal_unit_num,
                                                             uint64_t dynamic_unit_num, size_t spill_threshold_bytes)
    : ctx_(ctx), params_(params), agg_(ctx, params), normal_row_limit_(row_limit_unit * normal_unit_num),
      dynamic_row_limit_(row_limit_unit * dynamic_unit_num), row_limit_unit_(row_limit_unit),
      max_dynamic_row_limit_(row_limit_unit * MAX_DYNAMIC_UNIT_LIMIT), spill_threshold_(spill_threshold_bytes) {
    if (params_.keys.empty()) throw Exception("auto pass through needs GROUP BY keys", ErrorCodes::LOGICAL_ERROR);
    header_ = agg_.convertToBlock(true).cloneEmpty();
}

// HashMap<UInt64, AggregateDataPtr>::getBufferSizeInBytes: 16-byte cells, grown to keep the
// load <= 1/2 (HashTableGrower: initial 256 cells, doubling)
size_t AutoPassThroughHashAggContext::hashMapBytes() const {
    const size_t g = agg_.size();
    size_t cells = 256;
    while (cells < 2 * g) cells *= 2;
    return cells * 16;
}

// the map's cells plus one aggregate-state record per group (the Arena's share)
size_t AutoPassThroughHashAggContext::revocableBytes() const {
    size_t state = 0;
    for (const auto &d : params_.aggregates) state += d.function == "sum" ? 16 : 8; // min / max / first_row: 8
    return hashMapBytes() + agg_.size() * state;
}

bool AutoPassThroughHashAggContext::tryMarkNeedSpill() {
    if (need_spill_) return true;
    if (agg_.size() == 0 || already_get_data_from_hash_table_) return false; // empty(): nothing to spill
    need_spill_ = true;
    return true;
}

// forceState (:86-90): a map marked for spill, or already handed over, takes no more rows
void AutoPassThroughHashAggContext::forceState() {
    if (need_spill_ || already_get_data_from_hash_table_) state_ = State::PassThrough;
}

void AutoPassThroughHashAggContext::trySwitchFromInitState() {
    if (hashMapBytes() > INIT_STATE_HASHMAP_THRESHOLD) state_ = State::Adjust;
}

void AutoPassThroughHashAggContext::trySwitchFromAdjustState(size_t total_rows, size_t hit_rows) {
    adjust_processed_rows_ += total_rows;
    adjust_hit_rows_ += hit_rows;
    if (adjust_processed_rows_ < normal_row_limit_) return;
    const double hit_rate = (double)adjust_hit_rows_ / (double)adjust_processed_rows_;
    if (hit_rate >= PreHashAggRateLimit) state_ = State::PreHashAgg;
    else if (hit_rate <= PassThroughRateLimit) state_ = State::PassThrough;
    else state_ = State::Selective;
    adjust_processed_rows_ = adjust_hit_rows_ = 0;
    if (state_ == State::Selective) buildLookup();
}

void AutoPassThroughHashAggContext::trySwitchBackAdjustState(size_t block_rows) {
    state_processed_rows_ += block_rows;
    const size_t limit = state_ == State::PreHashAgg ? normal_row_limit_ : dynamic_row_limit_;
    if (state_processed_rows_ < limit) return;
    if (state_ == State::PassThrough || state_ == State::Selective)
        dynamic_row_limit_ = std::min(max_dynamic_row_limit_, dynamic_row_limit_ * 2);
    state_ = State::Adjust;
    state_processed_rows_ = 0;
    lookup_.reset();
}

// the map's key tuples as a join build side: a LeftOuterSemi probe then says "key is in the
// map".  One key: the single-key join (NULL keys are not inserted; the NULL group is tracked in
// lookup_has_null_).  Several keys: the multi-key join on the full tuple under the aggregator's
// collators; a tuple holding a NULL never matches, so such rows pass through (always safe: the
// second stage merges them), and the map never grows in the Selective state.
void AutoPassThroughHashAggContext::buildLookup() {
    Block keys = agg_.convertToBlock(true);
    Block kb;
    for (const auto &name : params_.keys) kb.insert(keys.getByName(name));
    if (params_.keys.size() == 1) {
        lookup_ = std::make_unique<Join>(ctx_, JoinKind::LeftOuterSemi, params_.keys[0], params_.keys[0]);
    } else {
        std::vector<int> coll;
        if (params_.collators.size() == params_.keys.size()) coll = params_.collators;
        lookup_ = std::make_unique<Join>(ctx_, JoinKind::LeftOuterSemi, params_.keys, params_.keys,
                                         (int64_t)kb.rows(), coll);
    }
    lookup_->setMatchHelperName("__in_map");
    lookup_->insertFromBlock(kb); // NULL keys are not inserted: tracked separately
    lookup_->finishOneBuild();
    lookup_has_null_ = false;
    const auto &k = kb.getByName(params_.keys[0]);
    if (params_.keys.size() == 1 && k.column->nullmap) {
        std::vector<uint8_t> nm = toHostNullMap(ctx_, *k.column);
        for (uint8_t x : nm) lookup_has_null_ |= x != 0;
    }
}

Block AutoPassThroughHashAggContext::getPassThroughBlock(const Block &block) const {
    const size_t n = block.rows();
    Block out;
    for (const auto &name : params_.keys) { // every GROUP BY key, as the second stage merges on the tuple
        const auto &kc = block.getByName(name);
        out.insert({kc.column, kc.column->type, name});
    }
    for (size_t i = 0; i < params_.aggregates.size(); ++i) {
        const AggregateDescription &d = params_.aggregates[i];
        const DataType rt = header_.getByName(d.column_name).type;
        auto c = std::make_shared<IColumn>();
        c->rows = n;
        if (d.function == "count" && d.argument_names.empty()) { // count() -> 1
            DataType u64;
            u64.type = TFG_UINT64;
            ColumnPtr one = materialize(ctx_, makeConstColumn(u64, 1, n));
            out.insert({one, u64, d.column_name});
            continue;
        }
        ColumnPtr arg = materialize(ctx_, block.getByName(d.argument_names[0]).column);
        if (d.function == "min" || d.function == "max" || d.function == "first_row") { // the value itself
            auto v = std::make_shared<IColumn>(*arg); // shares the argument's buffers
            v->type = rt;
            if (rt.nullable && !v->nullmap) {
                v->nullmap = std::make_shared<DeviceBuffer>(ctx_, std::max<size_t>(n, 1));
                const std::vector<uint8_t> zero(std::max<size_t>(n, 1), 0);
                check(tfg_upload(ctx_.raw(), v->nullmap->data(), zero.data(), zero.size()), "tfg_upload");
            }
            out.insert({v, v->type, d.column_name});
            continue;
        }
        c->data = std::make_shared<DeviceBuffer>(ctx_, std::max<size_t>(n, 1) * std::max<size_t>(rt.width(), 1));
        if (d.function == "count") { // count(x) -> 1, 0 where x is NULL
            c->type.type = TFG_UINT64;
            if (!arg->nullmap) {
                ColumnPtr one = materialize(ctx_, makeConstColumn(c->type, 1, n));
                out.insert({one, c->type, d.column_name});
                continue;
            }
            DeviceBuffer notnull(ctx_, std::max<size_t>(n, 1));
            const uint8_t zero = 0;
            if (n) {
                check(tfg_mask_logic(ctx_.raw(), TFG_NOT, arg->nullPtr(), nullptr, (int64_t)n, (uint8_t *)notnull.data()),
                      "tfg_mask_logic");
                check(tfg_arith(ctx_.raw(), TFG_PLUS, TFG_UINT8, notnull.data(), 0, 0, TFG_UINT8, &zero, 1, 0, TFG_UINT64, 0,
                                (int64_t)n, c->data->data()),
                      "tfg_arith");
            }
            ctx_.sync();
            out.insert({c, c->type, d.column_name});
            continue;
        }
        // sum(x) -> x widened to the sum's result type; NULL rows stay NULL
        c->type = rt;
        const uint64_t zero[2] = {0, 0};
        if (n)
            check(tfg_arith(ctx_.raw(), TFG_PLUS, arg->type.type, arg->dataPtr(), 0, arg->type.scale, arg->type.type, zero,
                            1, arg->type.scale, rt.type, rt.scale, (int64_t)n, c->data->data()),
                  "tfg_arith");
        if (rt.nullable) {
            c->nullmap = std::make_shared<DeviceBuffer>(ctx_, std::max<size_t>(n, 1));
            if (n) check(tfg_copy(ctx_.raw(), c->nullmap->data(), arg->nullPtr(), n), "tfg_copy");
        }
        ctx_.sync();
        out.insert({c, c->type, d.column_name});
    }
    return out;
}

void AutoPassThroughHashAggContext::onBlock(const Block &block, bool force_streaming) {
    if (!block || block.rows() == 0) return;
    const size_t rows = block.rows();
    if (force_streaming) {
        buffer_.push_back(getPassThroughBlock(block));
        pass_through_rows_ += rows;
        return;
    }
    forceState();
    switch (state_) {
    case State::Init:
        agg_.executeOnBlock(block);
        aggregated_rows_ += rows;
        trySwitchFromInitState();
        break;
    case State::Adjust: {
        // executeOnBlockCollectHitRate: every row either creates a group or hits one
        const size_t before = agg_.size();
        agg_.executeOnBlock(block);
        aggregated_rows_ += rows;
        const size_t created = agg_.size() - before;
        trySwitchFromAdjustState(rows, rows - created);
        break;
    }
    case State::PreHashAgg:
        agg_.executeOnBlock(block);
        aggregated_rows_ += rows;
        trySwitchBackAdjustState(rows);
        break;
    case State::PassThrough:
        buffer_.push_back(getPassThroughBlock(block));
        pass_through_rows_ += rows;
        trySwitchBackAdjustState(rows);
        break;
    case State::Selective: {
        // executeOnBlockOnlyLookup: rows whose key is in the map are aggregated (the map does
        // not grow), the others pass through
        if (!lookup_) buildLookup();
        Block kb;
        for (const auto &name : params_.keys) kb.insert(block.getByName(name));
        Block probed = lookup_->joinBlock(kb);
        ColumnPtr m = materialize(ctx_, probed.getByName("__in_map").column);
        auto hit = std::make_shared<IColumn>();
        hit->type.type = TFG_UINT8;
        hit->rows = rows;
        hit->data = m->data;
        if (m->nullmap) { // a NULL match (NULL in the probe tuple) is not a hit
            auto h2 = std::make_shared<IColumn>(*hit);
            h2->data = std::make_shared<DeviceBuffer>(ctx_, rows);
            DeviceBuffer notnull(ctx_, std::max<size_t>(rows, 1));
            check(tfg_mask_logic(ctx_.raw(), TFG_NOT, m->nullPtr(), nullptr, (int64_t)rows, (uint8_t *)notnull.data()),
                  "tfg_mask_logic");
            check(tfg_mask_logic(ctx_.raw(), TFG_AND, (const uint8_t *)hit->dataPtr(), (const uint8_t *)notnull.data(),
                                 (int64_t)rows, (uint8_t *)h2->data->data()),
                  "tfg_mask_logic");
            ctx_.sync();
            hit = h2;
        }
        ColumnPtr key = materialize(ctx_, block.getByName(params_.keys[0]).column);
        if (params_.keys.size() == 1 && lookup_has_null_ && key->nullmap) { // the NULL key's group is in the map too
            auto h2 = std::make_shared<IColumn>(*hit);
            h2->data = std::make_shared<DeviceBuffer>(ctx_, rows);
            check(tfg_mask_logic(ctx_.raw(), TFG_OR, (const uint8_t *)hit->dataPtr(), key->nullPtr(), (int64_t)rows,
                                 (uint8_t *)h2->data->data()),
                  "tfg_mask_logic");
            hit = h2;
        }
        auto miss = std::make_shared<IColumn>(*hit);
        miss->data = std::make_shared<DeviceBuffer>(ctx_, rows);
        check(tfg_mask_logic(ctx_.raw(), TFG_NOT, (const uint8_t *)hit->dataPtr(), nullptr, (int64_t)rows,
                             (uint8_t *)miss->data->data()),
              "tfg_mask_logic");
        ctx_.sync();
        const size_t before = agg_.size();
        agg_.executeOnBlock(block, hit);
        if (agg_.size() != before) throw Exception("Selective state grew the hash map", ErrorCodes::LOGICAL_ERROR);
        uint64_t nmiss = 0;
        check(tfg_count_mask(ctx_.raw(), (const uint8_t *)miss->dataPtr(), nullptr, (int64_t)rows, nullptr, &nmiss),
              "tfg_count_mask");
        aggregated_rows_ += rows - nmiss;
        if (nmiss) {
            Block pt = getPassThroughBlock(block);
            DataType u8;
            u8.type = TFG_UINT8;
            pt.insert({miss, u8, "__miss"});
            FilterTransformAction f(ctx_, pt.cloneEmpty(), nullptr, "__miss");
            FilterPtr none;
            f.transform(pt, none, false);
            pt.erase(pt.getPositionByName("__miss"));
            buffer_.push_back(pt);
            pass_through_rows_ += nmiss;
        }
        trySwitchBackAdjustState(rows);
        break;
    }
    }
    // after a block folded into the map: past the spill threshold the map is marked for spill
    if (spill_threshold_ && !need_spill_ && revocableBytes() > spill_threshold_) tryMarkNeedSpill();
}

Block AutoPassThroughHashAggContext::tryGetDataInAdvance() {
    // tryGetDataInAdvance (:92-104): a map marked for spill is handed over first, once
    if (need_spill_ && !already_get_data_from_hash_table_)
        if (Block m = getDataFromHashTable()) return m;
    if (buffer_head_ < buffer_.size()) {
        Block b = std::move(buffer_[buffer_head_++]);
        if (buffer_head_ == buffer_.size()) {
            buffer_.clear();
            buffer_head_ = 0;
        }
        return b;
    }
    return Block();
}

Block AutoPassThroughHashAggContext::getDataFromHashTable() {
    if (already_get_data_from_hash_table_) return Block();
    already_get_data_from_hash_table_ = true;
    lookup_.reset();
    if (agg_.size() == 0) return Block();
    return agg_.convertToBlock(true);
}

} // namespace tfa
