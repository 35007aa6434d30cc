// codec.cpp — CHBlockChunkCodec / CHBlockChunkCodecV1 over the device codec (tfg_codec_*).
// Reference: Flash/Coprocessor/CHBlockChunkCodec.cpp:134-258, CHBlockChunkCodecV1.cpp:45-147,
// 370-583.  The host side only names columns and types; the bytes stay on the device.
#include <cstdio>

#include "tfa_host.h"

namespace tfa {

DevicePacket encodeBlockPacket(Context &ctx, const Block &block, int version) {
    const size_t rows = block.rows();
    std::vector<ColumnPtr> keep;
    std::vector<std::string> types;
    std::vector<tfg_codec_column> cols(block.columns());
    for (size_t i = 0; i < block.columns(); ++i) {
        const auto &c = block.safeGetByPosition(i);
        // header-only columns (cloneEmpty) carry no column: only their type is written
        ColumnPtr col = !c.column ? nullptr : c.column->isColumnConst() ? materialize(ctx, c.column) : c.column;
        keep.push_back(col);
        types.push_back((col ? col->type : c.type).getName());
    }
    for (size_t i = 0; i < block.columns(); ++i) {
        const auto &c = block.safeGetByPosition(i);
        const ColumnPtr &col = keep[i];
        cols[i].name = c.name.c_str();
        cols[i].type_name = types[i].c_str();
        cols[i].data = col ? col->dataPtr() : nullptr;
        cols[i].offsets = col && col->offsets ? (const uint64_t *)col->offsets->data() : nullptr;
        cols[i].nullmap = col ? col->nullPtr() : nullptr;
    }
    size_t bytes = 0;
    check(tfg_codec_encode(ctx.raw(), version, (int)cols.size(), cols.data(), (int64_t)rows, nullptr, 0, &bytes),
          "tfg_codec_encode");
    DevicePacket p;
    if (!bytes) return p;
    p.buf = std::make_shared<DeviceBuffer>(ctx, bytes);
    check(tfg_codec_encode(ctx.raw(), version, (int)cols.size(), cols.data(), (int64_t)rows, (uint8_t *)p.buf->data(),
                           bytes, &p.bytes),
          "tfg_codec_encode");
    return p;
}

static DataType typeFromWire(int t, int nullable, const char *name) {
    DataType d;
    d.type = t == TFG_STRING ? DataType::TYPE_STRING : t;
    d.nullable = nullable != 0;
    const char *dec = strstr(name, "Decimal(");
    int prec = 0, scale = 0;
    if (dec && sscanf(dec, "Decimal(%d,%d)", &prec, &scale) == 2) {
        d.scale = scale;
        d.prec = prec;
    }
    return d;
}

Block decodeBlockPacket(Context &ctx, const Block &header, const uint8_t *packet, size_t bytes, int version) {
    if (!bytes) return Block(); // decodeImpl: eof -> empty Block
    tfg_codec_packet *p = nullptr;
    check(tfg_codec_decode(ctx.raw(), version, packet, bytes, &p), "tfg_codec_decode");
    struct Guard {
        tfg_codec_packet *p;
        ~Guard() { tfg_codec_packet_destroy(p); }
    } guard{p};
    int ncols = 0;
    int64_t rows = 0;
    check(tfg_codec_packet_info(p, &ncols, &rows), "tfg_codec_packet_info");
    if (header && header.columns() != (size_t)ncols) // CodecUtils::checkColumnSize
        throw Exception("CHBlockChunkCodec: column count mismatch, expect " + std::to_string(header.columns()) +
                            ", actual " + std::to_string(ncols),
                        ErrorCodes::LOGICAL_ERROR);
    Block out;
    for (int i = 0; i < ncols; ++i) {
        char name[256], tname[256];
        int t = 0, nl = 0;
        uint64_t chars = 0;
        check(tfg_codec_column_info(p, i, name, sizeof(name), tname, sizeof(tname), &t, &nl, &chars),
              "tfg_codec_column_info");
        auto c = std::make_shared<IColumn>();
        c->type = typeFromWire(t, nl, tname);
        c->rows = (size_t)rows;
        if (c->type.isString()) {
            c->chars = chars;
            c->data = std::make_shared<DeviceBuffer>(ctx, std::max<size_t>(chars, 1));
            c->offsets = std::make_shared<DeviceBuffer>(ctx, std::max<size_t>(rows, 1) * 8);
        } else {
            c->data = std::make_shared<DeviceBuffer>(ctx, std::max<size_t>(rows, 1) * c->type.width());
        }
        if (nl) c->nullmap = std::make_shared<DeviceBuffer>(ctx, std::max<size_t>(rows, 1));
        check(tfg_codec_column_read(p, i, c->data->data(), c->offsets ? (uint64_t *)c->offsets->data() : nullptr,
                                    c->nullmap ? (uint8_t *)c->nullmap->data() : nullptr),
              "tfg_codec_column_read");
        std::string cname = header ? header.safeGetByPosition(i).name : std::string(name);
        out.insert(ColumnWithTypeAndName{c, c->type, cname});
    }
    ctx.sync();
    return out;
}

DevicePacket CHBlockChunkCodecV1::encode(const Block &block) {
    DevicePacket p = encodeBlockPacket(ctx_, block, TFG_CODEC_V1);
    if (!p.empty()) {
        encoded_rows += block.rows();
        original_size += p.bytes;
    }
    return p;
}

DevicePacket CHBlockChunkCodecV1::encode(const std::vector<Block> &blocks) {
    std::vector<Block> nonempty;
    for (const Block &b : blocks)
        if (b && b.rows()) nonempty.push_back(b);
    if (nonempty.empty()) return DevicePacket();
    return encode(concatenateBlocks(ctx_, nonempty));
}

Block CHBlockChunkCodecV1::decode(Context &ctx, const Block &header, const DevicePacket &packet) {
    return decodeBlockPacket(ctx, header, packet.buf ? (const uint8_t *)packet.buf->data() : nullptr, packet.bytes,
                             TFG_CODEC_V1);
}

DevicePacket CHBlockChunkCodec::encode(const Block &block) { return encodeBlockPacket(ctx_, block, TFG_CODEC_CHBLOCK); }

Block CHBlockChunkCodec::decode(const DevicePacket &packet) const {
    return decodeBlockPacket(ctx_, header_, packet.buf ? (const uint8_t *)packet.buf->data() : nullptr, packet.bytes,
                             TFG_CODEC_CHBLOCK);
}

} // namespace tfa
