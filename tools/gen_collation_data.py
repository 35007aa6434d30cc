#!/usr/bin/env python3
"""Generates the collation weight data for the device code and the oracle:

collation_data.h  utf8mb4_general_ci, from the reference's GeneralCI::weight_lut
                  (dbms/src/TiDB/Collation/CollationLUT.cpp:18-359, MySQL's general_ci weights: one
                  16-bit weight per BMP code point, most planes the identity);
uca_data.h        utf8mb4_unicode_ci (UCA 4.0.0) and utf8mb4_0900_ai_ci (UCA 9.0.0), from
                  UnicodeCI::weight_lut_0400 / weight_lut_0900 (CollationLUT.cpp:361-249872: up to
                  four 16-bit weights per code point packed in a u64, 0xFFFD = "long weight") and the
                  long weights with their code points (Collator.cpp:468-523, 729-780, 818-870).

The table is re-encoded, not copied: the code points whose weight differs from the code point
become runs [first, last] with either a constant weight offset (weight = code + delta, e.g.
a-z -> A-Z) or one weight for the whole run (e.g. the accented forms of a letter -> the letter).
Lookups binary-search the runs; code points outside every run weigh themselves, and code points
past the BMP weigh 0xFFFD (GeneralCICollator::weight, Collator.h:403-407).

usage: python3 tools/gen_collation_data.py   (reads /root/reference; run in the build container)
"""
import os
import re

REF = "/root/reference/dbms/src/TiDB/Collation/CollationLUT.cpp"
REF_COLL = "/root/reference/dbms/src/TiDB/Collation/Collator.cpp"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUTS = [os.path.join(ROOT, "tiflash_amd", "csrc", "collation_data.h"), os.path.join(ROOT, "oracle", "collation_data.h")]
UCA_OUTS = [os.path.join(ROOT, "tiflash_amd", "csrc", "uca_data.h"), os.path.join(ROOT, "oracle", "uca_data.h")]
NUM = re.compile(r"0x[0-9A-Fa-f]+|\b\d+\b")


def planes():
    lines = open(REF).read().split("\n")
    out, cur, vals = {}, None, []
    for line in lines:
        m = re.match(r"#define PLANE_([0-9A-F]{2})\b", line)
        if m:
            if cur is not None:
                out[cur] = vals
            cur, vals = int(m.group(1), 16), []
            continue
        if line.startswith("#define CONCAT"):
            break
        if cur is not None:
            vals += [int(x, 16) for x in re.findall(r"0x[0-9A-Fa-f]+", line)]
    out[cur] = vals
    for p, v in out.items():
        assert len(v) == 256, (p, len(v))
    return out


def runs(pl):
    w = list(range(65536))
    for p, v in pl.items():
        w[p << 8:(p << 8) + 256] = v
    res, c = [], 0
    while c < 65536:
        if w[c] == c:
            c += 1
            continue
        # the longer of: a constant-delta run, a constant-weight run
        d, e1 = w[c] - c, c
        while e1 + 1 < 65536 and w[e1 + 1] != e1 + 1 and w[e1 + 1] - (e1 + 1) == d:
            e1 += 1
        e2 = c
        while e2 + 1 < 65536 and w[e2 + 1] != e2 + 1 and w[e2 + 1] == w[c]:
            e2 += 1
        if e2 > e1:
            res.append((c, e2, 1, w[c]))
            c = e2 + 1
        else:
            res.append((c, e1, 0, d & 0xFFFF))
            c = e1 + 1
    # check the encoding reproduces every weight
    def look(x):
        for a, b, k, val in res:
            if a <= x <= b:
                return val if k else (x + (val - 65536 if val >= 32768 else val)) & 0xFFFF
        return x
    assert all(look(x) == w[x] for x in range(65536))
    return res


def uca_table(name, size):
    """the values of `extern const std::array<uint64_t, ...> <name> = { ... };`"""
    text = open(REF).read()
    i = text.index(name)
    body = text[text.index("{", i) + 1:text.index("};", i)]
    body = re.sub(r"//[^\n]*|/\*.*?\*/", "", body)  # comments
    vals = [int(x, 16) if x.startswith("0x") else int(x) for x in NUM.findall(body)]
    assert len(vals) <= size, (name, len(vals), size)
    return vals + [0] * (size - len(vals))  # std::array aggregate init: the rest are zero


def delta_runs(t):
    """[(start, count, base, delta)]: t[start + k] = base + k * delta (mod 2^64)"""
    out, i = [], 0
    while i < len(t):
        d = (t[i + 1] - t[i]) % (1 << 64) if i + 1 < len(t) else 0
        j = i + 1
        while j < len(t) and (t[j] - t[j - 1]) % (1 << 64) == d:
            j += 1
        out.append((i, j - i, t[i], d))
        i = j
    exp = []
    for st, n, b, d in out:
        exp += [(b + k * d) % (1 << 64) for k in range(n)]
    assert exp == t
    return out


def uca_long(tag):
    """{code point, first, second} of the long weights of UCA <tag> ('0400' / '0900')"""
    text = open(REF_COLL).read()
    i = text.index("weight_lut_long_%s\n" % tag if False else "std::array<long_weight")
    i = text.index("weight_lut_long_" + tag, i)
    body = text[text.index("{", i) + 1:text.index("};", i)]
    ws = [(int(a, 16), int(b, 16)) for a, b in re.findall(r"long_weight\{(0x[0-9A-Fa-f]+),\s*(0x[0-9A-Fa-f]+)\}", body)]
    j = text.index("Unicode%s::weightLutLongMap(Rune r)" % tag)
    k = text.index("default:", j)
    cases = re.findall(r"case (0x[0-9A-Fa-f]+):\s*return UnicodeCI::weight_lut_long_%s\[(\d+)\];" % tag, text[j:k])
    assert cases and all(int(ix) < len(ws) for _, ix in cases), tag
    return [(int(cp, 16),) + ws[int(ix)] for cp, ix in cases]


def write_uca():
    parts = ["// uca_data.h — utf8mb4_unicode_ci (UCA 4.0.0) and utf8mb4_0900_ai_ci (UCA 9.0.0) weights",
             "// (GENERATED by tools/gen_collation_data.py; do not edit).  Each weight table is stored as",
             "// runs {first code point, count, base, delta}: weight(first + k) = base + k * delta (mod 2^64);",
             "// the runs cover [0, TFG_UCAxxxx_SIZE) in order.  0xFFFD marks a long weight, listed in",
             "// TFG_UCAxxxx_LONG as {code point, first, second}.",
             "#pragma once", "#include <stdint.h>", ""]
    for tag, size in (("0400", 256 * 256 + 1), ("0900", 0x2CEA1)):
        rs = delta_runs(uca_table("weight_lut_" + tag, size))
        lw = uca_long(tag)
        parts.append("#define TFG_UCA%s_SIZE %d" % (tag, size))
        parts.append("#define TFG_UCA%s_NRUNS %d" % (tag, len(rs)))
        parts.append("#define TFG_UCA%s_RUNS_INIT \\" % tag)
        parts.append(", \\\n".join("    {%d, %d, 0x%xull, 0x%xull}" % r for r in rs))
        parts.append("")
        parts.append("#define TFG_UCA%s_NLONG %d" % (tag, len(lw)))
        parts.append("#define TFG_UCA%s_LONG_INIT \\" % tag)
        parts.append(", \\\n".join("    {0x%x, 0x%xull, 0x%xull}" % w for w in lw))
        parts.append("")
    text = "\n".join(parts)
    for o in UCA_OUTS:
        with open(o, "w") as f:
            f.write(text)
    print("uca_data.h", len(text), "bytes")


def main():
    write_uca()
    rs = runs(planes())
    body = ", \\\n".join("    {%d, %d, %d}" % (a, b, (k << 16) | v) for a, b, k, v in rs)
    text = f"""// collation_data.h — utf8mb4_general_ci weights (GENERATED by tools/gen_collation_data.py; do not edit).
// Runs of BMP code points whose weight is not the code point itself: {{first, last, kind << 16 | value}}
// with kind 0: weight = code + (int16_t)value, kind 1: weight = value.  Sorted by first.
#pragma once
#include <stdint.h>

#define TFG_GCI_RUNS {len(rs)}
#define TFG_GCI_RUNS_INIT \\
{body}
"""
    for o in OUTS:
        with open(o, "w") as f:
            f.write(text)
    print(len(rs), "runs")


if __name__ == "__main__":
    main()
