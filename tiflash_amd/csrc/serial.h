// serial.h — the `serialized` GROUP BY method's key dictionary (serial.hip).
//
// Aggregator::chooseAggregationMethod (Interpreters/Aggregator.cpp:394-537) falls back to
// AggregationMethodSerialized (HashMethodSerialized, Common/ColumnsHashing.h:578-629) when the key
// tuple cannot be packed: String keys together with other keys, fixed keys wider than keys256,
// nullable key tuples past nullable_keys256.  The reference serialises each row's key tuple into
// an arena and hashes the bytes.  Here a device dictionary maps each distinct key tuple to a dense
// group id: rows are fingerprinted, the fingerprint finds (or claims) a slot in an open-addressing
// table, the first row of a new slot writes the tuple's serialised bytes into a key arena, and every
// row is verified byte-for-byte against its slot's arena entry.  Rows whose fingerprint collided
// with a different tuple retry with the next seed, so a collision costs a retry, never a wrong group.
// The aggregation itself then runs on the UInt32 group ids through the fixed-key path.
#pragma once

#include "common.h"

namespace tfg {

struct SerialDict;

// nkeys 1..8 key columns (tfg_type; TFG_STRING by collator's sort key).
int serial_dict_create(Ctx *ctx, int nkeys, const int *key_types, const int *key_collators, SerialDict **out);
void serial_dict_destroy(SerialDict *d);
void serial_dict_reset(SerialDict *d);
uint64_t serial_dict_groups(const SerialDict *d);
// out_gid[r] = the dense group id of row r's key tuple (new tuples get new ids); rows with
// mask[r] == 0 get 0 and create nothing.  out_gid: n device u32.
int serial_dict_assign(SerialDict *d, const void *const *key_cols, const uint64_t *const *key_offsets,
                       const uint8_t *const *key_nullmaps, const uint8_t *mask, int64_t n, uint32_t *out_gid);
// Writes the key columns of groups gid[0..G): fixed keys (width bytes each), String keys (chars
// with '\0' terminators + end offsets), null maps (optional).  String chars need
// out_chars[j] bytes per String key j (*out_chars_max = the largest); TFG_ERR_CAPACITY past
// chars_capacity (then nothing is written).
int serial_dict_unpack(SerialDict *d, const uint32_t *gid, uint64_t G, void *const *out_cols,
                       uint64_t *const *out_offsets, uint8_t *const *out_nullmaps, uint64_t chars_capacity,
                       uint64_t *out_chars_max);

} // namespace tfg
