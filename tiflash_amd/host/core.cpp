// core.cpp — errors, device context, columns and blocks of the host layer (tfa_host.h).
#include <algorithm>
#include <cstring>

#include "tfa_host.h"

namespace tfa {

void check(int status, const char *what) {
    if (status == TFG_OK) return;
    int code = ErrorCodes::LOGICAL_ERROR;
    switch (status) {
    case TFG_ERR_INVALID_ARG: code = ErrorCodes::BAD_ARGUMENTS; break;
    case TFG_ERR_SIZE_MISMATCH: code = ErrorCodes::SIZES_OF_COLUMNS_DOESNT_MATCH; break;
    case TFG_ERR_ILLEGAL_TYPE: code = ErrorCodes::ILLEGAL_TYPE_OF_ARGUMENT; break;
    case TFG_ERR_NOT_IMPLEMENTED: code = ErrorCodes::NOT_IMPLEMENTED; break;
    case TFG_ERR_OOM: code = ErrorCodes::CANNOT_ALLOCATE_MEMORY; break;
    case TFG_ERR_OVERFLOW: code = ErrorCodes::DECIMAL_OVERFLOW; break;
    default: break;
    }
    throw Exception(std::string(what) + ": " + tfg_last_error(), code);
}

Context::Context(int device) : device_(device) { check(tfg_ctx_create(device, nullptr, &ctx_), "tfg_ctx_create"); }
Context::~Context() {
    if (ctx_) tfg_ctx_destroy(ctx_);
}
void Context::sync() const { check(tfg_ctx_sync(ctx_), "tfg_ctx_sync"); }

DeviceBuffer::DeviceBuffer(Context &ctx, size_t bytes) : ctx_(ctx), bytes_(bytes) {
    check(tfg_buf_alloc(ctx.raw(), std::max<size_t>(bytes, 16), &ptr_), "tfg_buf_alloc");
}
DeviceBuffer::~DeviceBuffer() {
    if (ptr_) tfg_buf_free(ctx_.raw(), ptr_);
}

size_t DataType::width() const { return isString() ? 0 : tfg_type_width(type); }

int DataType::precision() const {
    if (prec > 0) return prec;
    switch (type) {
    case TFG_DECIMAL32: return 9;
    case TFG_DECIMAL64: return 18;
    case TFG_DECIMAL128: return 38;
    case TFG_DECIMAL256: return 65;
    default: return 0;
    }
}

DataType DataType::decimal(int p, int s, bool nullable) {
    if (p < 1 || p > 65 || s < 0 || s > p)
        throw Exception("Decimal(" + std::to_string(p) + "," + std::to_string(s) + ") is out of range",
                        ErrorCodes::BAD_ARGUMENTS);
    DataType d;
    d.type = p <= 9 ? TFG_DECIMAL32 : p <= 18 ? TFG_DECIMAL64 : p <= 38 ? TFG_DECIMAL128 : TFG_DECIMAL256;
    d.prec = p;
    d.scale = s;
    d.nullable = nullable;
    return d;
}

std::string DataType::getName() const {
    std::string n;
    switch (type) {
    case TFG_INT8: n = "Int8"; break;
    case TFG_INT16: n = "Int16"; break;
    case TFG_INT32: n = "Int32"; break;
    case TFG_INT64: n = "Int64"; break;
    case TFG_UINT8: n = "UInt8"; break;
    case TFG_UINT16: n = "UInt16"; break;
    case TFG_UINT32: n = "UInt32"; break;
    case TFG_UINT64: n = "UInt64"; break;
    case TFG_FLOAT32: n = "Float32"; break;
    case TFG_FLOAT64: n = "Float64"; break;
    case TFG_DECIMAL32:
    case TFG_DECIMAL64:
    case TFG_DECIMAL128:
    case TFG_DECIMAL256: n = "Decimal(" + std::to_string(precision()) + "," + std::to_string(scale) + ")"; break;
    case TYPE_STRING: n = "String"; break;
    default: n = "Unknown"; break;
    }
    return nullable ? "Nullable(" + n + ")" : n;
}

void Block::insert(size_t position, ColumnWithTypeAndName c) {
    if (position > data_.size())
        throw Exception("Position out of bound in Block::insert()", ErrorCodes::BAD_ARGUMENTS);
    data_.insert(data_.begin() + position, std::move(c));
}

void Block::erase(size_t position) {
    if (position >= data_.size())
        throw Exception("Position out of bound in Block::erase()", ErrorCodes::BAD_ARGUMENTS);
    data_.erase(data_.begin() + position);
}

size_t Block::rows() const {
    size_t r = 0;
    bool first = true;
    for (const auto &c : data_) {
        if (!c.column) continue;
        if (first) {
            r = c.column->rows;
            first = false;
        } else if (c.column->rows != r) {
            throw Exception("Sizes of columns doesn't match: " + c.name, ErrorCodes::SIZES_OF_COLUMNS_DOESNT_MATCH);
        }
    }
    return r;
}

bool Block::has(const std::string &name) const {
    for (const auto &c : data_)
        if (c.name == name) return true;
    return false;
}

size_t Block::getPositionByName(const std::string &name) const {
    for (size_t i = 0; i < data_.size(); ++i)
        if (data_[i].name == name) return i;
    throw Exception("Not found column " + name + " in block", ErrorCodes::NOT_FOUND_COLUMN_IN_BLOCK);
}

const ColumnWithTypeAndName &Block::getByName(const std::string &name) const { return data_[getPositionByName(name)]; }

ColumnWithTypeAndName &Block::safeGetByPosition(size_t i) {
    if (i >= data_.size()) throw Exception("Position out of bound in Block", ErrorCodes::BAD_ARGUMENTS);
    return data_[i];
}
const ColumnWithTypeAndName &Block::safeGetByPosition(size_t i) const {
    if (i >= data_.size()) throw Exception("Position out of bound in Block", ErrorCodes::BAD_ARGUMENTS);
    return data_[i];
}

Block Block::cloneEmpty() const {
    Block b;
    for (const auto &c : data_) b.insert({nullptr, c.type, c.name});
    return b;
}

// ---------------------------------------------------------------- host <-> device
BlockSelectivePtr makeSelective(Context &ctx, const std::vector<uint64_t> &rows) {
    auto s = std::make_shared<BlockSelective>();
    s->count = rows.size();
    s->rows = std::make_shared<DeviceBuffer>(ctx, std::max<size_t>(rows.size(), 1) * 8);
    if (!rows.empty()) check(tfg_upload(ctx.raw(), s->rows->data(), rows.data(), rows.size() * 8), "tfg_upload");
    return s;
}

ColumnPtr makeColumn(Context &ctx, DataType type, const void *values, size_t rows, const uint8_t *nullmap) {
    if (type.isString()) throw Exception("use makeStringColumn", ErrorCodes::BAD_ARGUMENTS);
    auto c = std::make_shared<IColumn>();
    c->type = type;
    c->rows = rows;
    const size_t bytes = rows * type.width();
    c->data = std::make_shared<DeviceBuffer>(ctx, bytes);
    check(tfg_upload(ctx.raw(), c->data->data(), values, bytes), "tfg_upload");
    if (nullmap || type.nullable) {
        c->type.nullable = true;
        c->nullmap = std::make_shared<DeviceBuffer>(ctx, rows);
        std::vector<uint8_t> zeros;
        if (!nullmap) zeros.assign(rows, 0);
        check(tfg_upload(ctx.raw(), c->nullmap->data(), nullmap ? nullmap : zeros.data(), rows), "tfg_upload");
    }
    return c;
}

ColumnPtr makeStringColumn(Context &ctx, const std::vector<std::string> &values, const uint8_t *nullmap) {
    auto c = std::make_shared<IColumn>();
    c->type.type = DataType::TYPE_STRING;
    c->type.nullable = nullmap != nullptr;
    c->rows = values.size();
    std::vector<uint8_t> chars;
    std::vector<uint64_t> offs(values.size());
    for (size_t i = 0; i < values.size(); ++i) {
        chars.insert(chars.end(), values[i].begin(), values[i].end());
        chars.push_back(0);
        offs[i] = chars.size();
    }
    c->chars = chars.size();
    c->data = std::make_shared<DeviceBuffer>(ctx, chars.size());
    c->offsets = std::make_shared<DeviceBuffer>(ctx, offs.size() * 8);
    check(tfg_upload(ctx.raw(), c->data->data(), chars.data(), chars.size()), "tfg_upload");
    check(tfg_upload(ctx.raw(), c->offsets->data(), offs.data(), offs.size() * 8), "tfg_upload");
    if (nullmap) {
        c->nullmap = std::make_shared<DeviceBuffer>(ctx, values.size());
        check(tfg_upload(ctx.raw(), c->nullmap->data(), nullmap, values.size()), "tfg_upload");
    }
    return c;
}

ColumnPtr makeConstColumn(DataType type, uint64_t bits, size_t rows) {
    auto c = std::make_shared<IColumn>();
    c->type = type;
    c->rows = rows;
    c->is_const = true;
    c->const_value = bits;
    return c;
}

ColumnPtr materialize(Context &ctx, const ColumnPtr &c) {
    if (!c->is_const) return c;
    if (c->type.isString() || c->type.width() > 8)
        throw Exception("materialize: constant of this type", ErrorCodes::NOT_IMPLEMENTED);
    const size_t w = c->type.width();
    std::vector<uint8_t> host(c->rows * w);
    for (size_t i = 0; i < c->rows; ++i) memcpy(host.data() + i * w, &c->const_value, w);
    DataType t = c->type;
    t.nullable = false;
    return makeColumn(ctx, t, host.data(), c->rows);
}

std::vector<uint8_t> toHostBytes(Context &ctx, const IColumn &c) {
    if (c.is_const) {
        const size_t w = c.type.width();
        std::vector<uint8_t> out(c.rows * w);
        for (size_t i = 0; i < c.rows; ++i) memcpy(out.data() + i * w, &c.const_value, w);
        return out;
    }
    const size_t bytes = c.type.isString() ? c.chars : c.rows * c.type.width();
    std::vector<uint8_t> out(bytes);
    if (bytes) check(tfg_download(ctx.raw(), out.data(), c.dataPtr(), bytes), "tfg_download");
    return out;
}

std::vector<uint8_t> toHostNullMap(Context &ctx, const IColumn &c) {
    std::vector<uint8_t> out(c.rows, 0);
    if (c.nullmap && c.rows) check(tfg_download(ctx.raw(), out.data(), c.nullmap->data(), c.rows), "tfg_download");
    return out;
}

std::vector<std::string> toHostStrings(Context &ctx, const IColumn &c) {
    if (!c.type.isString()) throw Exception("not a String column", ErrorCodes::ILLEGAL_TYPE_OF_ARGUMENT);
    std::vector<uint8_t> chars = toHostBytes(ctx, c);
    std::vector<uint64_t> offs(c.rows);
    if (c.rows) check(tfg_download(ctx.raw(), offs.data(), c.offsets->data(), c.rows * 8), "tfg_download");
    std::vector<std::string> out(c.rows);
    uint64_t prev = 0;
    for (size_t i = 0; i < c.rows; ++i) {
        out[i].assign((const char *)chars.data() + prev, offs[i] - prev - 1);
        prev = offs[i];
    }
    return out;
}

Block concatenateBlocks(Context &ctx, const std::vector<Block> &blocks) {
    if (blocks.empty()) return Block();
    if (blocks.size() == 1) return blocks[0];
    Block out;
    const Block &first = blocks[0];
    for (size_t j = 0; j < first.columns(); ++j) {
        const auto &proto = first.safeGetByPosition(j);
        size_t rows = 0, chars = 0;
        bool any_null = false;
        for (const auto &b : blocks) {
            const IColumn &c = *b.safeGetByPosition(j).column;
            rows += c.rows;
            chars += c.chars;
            any_null |= c.nullmap != nullptr;
        }
        auto col = std::make_shared<IColumn>();
        col->type = proto.column->type;
        col->rows = rows;
        if (col->type.isString()) {
            col->chars = chars;
            col->data = std::make_shared<DeviceBuffer>(ctx, chars);
            col->offsets = std::make_shared<DeviceBuffer>(ctx, rows * 8);
            size_t r0 = 0, c0 = 0;
            for (const auto &b : blocks) {
                const IColumn &c = *b.safeGetByPosition(j).column;
                check(tfg_copy(ctx.raw(), (char *)col->data->data() + c0, c.dataPtr(), c.chars), "tfg_copy");
                // offsets of this piece rebased by the chars before it (an arithmetic kernel)
                const uint64_t base = c0;
                if (c.rows)
                    check(tfg_arith(ctx.raw(), TFG_PLUS, TFG_UINT64, c.offsets->data(), 0, 0, TFG_UINT64, &base, 1, 0,
                                    TFG_UINT64, 0, (int64_t)c.rows, (uint64_t *)col->offsets->data() + r0),
                          "tfg_arith");
                r0 += c.rows;
                c0 += c.chars;
            }
        } else {
            ColumnPtr keep;
            const size_t w = col->type.width();
            col->data = std::make_shared<DeviceBuffer>(ctx, rows * w);
            size_t r0 = 0;
            for (const auto &b : blocks) {
                ColumnPtr c = materialize(ctx, b.safeGetByPosition(j).column);
                check(tfg_copy(ctx.raw(), (char *)col->data->data() + r0 * w, c->dataPtr(), c->rows * w), "tfg_copy");
                r0 += c->rows;
            }
        }
        if (any_null) {
            col->type.nullable = true;
            col->nullmap = std::make_shared<DeviceBuffer>(ctx, rows);
            size_t r0 = 0;
            for (const auto &b : blocks) {
                const IColumn &c = *b.safeGetByPosition(j).column;
                if (c.nullmap) {
                    check(tfg_copy(ctx.raw(), (char *)col->nullmap->data() + r0, c.nullmap->data(), c.rows), "tfg_copy");
                } else if (c.rows) {
                    check(tfg_memset(ctx.raw(), (char *)col->nullmap->data() + r0, 0, c.rows), "tfg_memset");
                }
                r0 += c.rows;
            }
        }
        out.insert({col, col->type, proto.name});
    }
    ctx.sync();
    return out;
}

ColumnPtr gatherColumn(Context &ctx, const IColumn &src, const uint32_t *perm_dev, size_t n, bool make_nullable) {
    auto col = std::make_shared<IColumn>();
    col->type = src.type;
    col->rows = n;
    const int w = (int)src.type.width();
    if (src.is_const) {
        col->is_const = true;
        col->const_value = src.const_value;
        return col;
    }
    if (src.type.isString()) { // offsets, then the chars they need
        col->offsets = std::make_shared<DeviceBuffer>(ctx, std::max<size_t>(n, 1) * 8);
        uint64_t chars = 0;
        check(tfg_gather_string(ctx.raw(), perm_dev, (int64_t)n, (const uint8_t *)src.dataPtr(),
                                (const uint64_t *)src.offsets->data(), (uint64_t *)col->offsets->data(), nullptr, 0,
                                &chars),
              "tfg_gather_string");
        col->chars = chars;
        col->data = std::make_shared<DeviceBuffer>(ctx, std::max<uint64_t>(chars, 1));
        if (n)
            check(tfg_gather_string(ctx.raw(), perm_dev, (int64_t)n, (const uint8_t *)src.dataPtr(),
                                    (const uint64_t *)src.offsets->data(), (uint64_t *)col->offsets->data(),
                                    (uint8_t *)col->data->data(), chars, &chars),
                  "tfg_gather_string");
    } else {
        col->data = std::make_shared<DeviceBuffer>(ctx, n * w);
        const void *in[1] = {src.dataPtr()};
        void *out[1] = {col->data->data()};
        if (n) check(tfg_gather(ctx.raw(), perm_dev, (int64_t)n, 1, in, &w, out), "tfg_gather");
    }
    if (src.nullmap || make_nullable) {
        col->type.nullable = true;
        col->nullmap = std::make_shared<DeviceBuffer>(ctx, n);
        uint8_t *nm = (uint8_t *)col->nullmap->data();
        if (src.nullmap) {
            const int w1 = 1;
            const void *ni[1] = {src.nullmap->data()};
            void *no[1] = {nm};
            if (n) check(tfg_gather(ctx.raw(), perm_dev, (int64_t)n, 1, ni, &w1, no), "tfg_gather");
        }
        if (make_nullable && n) {
            // rows without a partner (perm == 0xFFFFFFFF) are NULL
            const uint32_t none = 0xFFFFFFFFu;
            DeviceBuffer unmatched(ctx, n);
            check(tfg_cmp_const(ctx.raw(), TFG_UINT32, perm_dev, nullptr, (int64_t)n, TFG_EQ, TFG_UINT32, &none,
                                (uint8_t *)unmatched.data()),
                  "tfg_cmp_const");
            if (src.nullmap)
                check(tfg_mask_logic(ctx.raw(), TFG_OR, nm, (const uint8_t *)unmatched.data(), (int64_t)n, nm),
                      "tfg_mask_logic");
            else
                check(tfg_copy(ctx.raw(), nm, unmatched.data(), n), "tfg_copy");
            ctx.sync();
        }
    }
    return col;
}

} // namespace tfa
