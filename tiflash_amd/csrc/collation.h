// collation.h — String sort keys of the case-insensitive collators on the device.
//
// Reference: GeneralCICollator::sortKey = convertImpl<false, true> (TiDB/Collation/Collator.cpp:
// 416-455): right-trim ' ' (RightTrim, CollatorCompare.h:56-61), decode UTF-8 (decodeUtf8Char,
// Collator.cpp:43-74, no validation), and emit each character's 16-bit weight big-endian
// (GeneralCICollator::weight, Collator.h:403-407: 0xFFFD past the BMP, else weight_lut).
// The UCA collators (utf8mb4_unicode_ci = UCACICollator<Unicode0400, padding>, utf8mb4_0900_ai_ci
// = UCACICollator<Unicode0900, no padding>; sortKey = convertImpl, Collator.cpp:580-629) skip
// zero-weight characters and write each character's weight words (one or two u64 of 16-bit
// chunks, low chunk first, each big-endian: writeResult, Collator.h:336-344).
// Every consumer of a String key under such a collator (weak hash, GROUP BY keys, join keys)
// hashes / compares the sort key, so the key column is collated once into a sort-key column in
// the ColumnString layout (bytes + '\0' per row, UInt64 end offsets) and the byte-wise code
// path runs on that column.
#pragma once
#include "common.h"

namespace tfg {

inline bool collator_transforms(int collator) {
    return collator == TFG_COLLATOR_GENERAL_CI || collator == TFG_COLLATOR_UNICODE_CI ||
           collator == TFG_COLLATOR_UCA0900_AI_CI;
}
inline bool collator_known(int collator) {
    return collator >= TFG_COLLATOR_NONE && collator <= TFG_COLLATOR_UCA0900_AI_CI;
}

// A collated column in the context's call arena (DevArena, common.h), held until the object dies.
struct CollatedStrings {
    Ctx *ctx = nullptr;
    uint8_t *chars = nullptr;
    uint64_t *scan = nullptr; // n + 1 start offsets; offsets() = scan + 1 = end offsets
    int64_t rows = 0;
    uint64_t bytes = 0; // sort-key bytes in `chars` (every row's key ends before it)
    const uint64_t *offsets() const { return scan + 1; }
    CollatedStrings() = default;
    CollatedStrings(const CollatedStrings &) = delete;
    CollatedStrings &operator=(const CollatedStrings &) = delete;
    ~CollatedStrings();
};

// Sort keys of rows sel[i] (sel32 / sel64; both null: rows 0..n-1) of a ColumnString under
// `collator` (collator_transforms).  NULL rows (nullmap) get an empty key.  whole: the sort key of
// the row with its terminating '\0' and without the padding trim (collator->compare over
// getDataAtWithTerminatingZero, as SingleValueDataString compares min / max candidates).
int collate_strings(Ctx *ctx, int collator, const uint8_t *chars, const uint64_t *offsets, const uint8_t *nullmap,
                    const uint32_t *sel32, const uint64_t *sel64, int64_t n, CollatedStrings &out, bool whole = false);

} // namespace tfg
