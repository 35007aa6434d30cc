// test_host.cpp — tests of the C++ host operators (tiflash_amd/host) on the GPU, written like the
// reference's gtests: the known answers of gtest_aggregation_executor.cpp (GroupBy),
// gtest_join_executor.cpp (SimpleJoin), gtest_mpp_exchange_writer.cpp (1024 rows per partition)
// and gtest_filter_executor.cpp, read from tests/golden/reference_cases.json, plus randomized
// cases checked against the CPU restatement (oracle/liboracle.so, test infrastructure).
//
// usage: test_host <repo_root> [test-name-substring]     (run by tests/test_gpu_host_cpp.py)
#include <cmath>
#include <cstdio>
#include <optional>
#include <random>
#include <cstdlib>
#include <fstream>
#include <map>
#include <random>
#include <set>
#include <sstream>

#include <arpa/inet.h>
#include <csignal>
#include <execinfo.h>
#include <netinet/in.h>
#include <sys/socket.h>
#include <unistd.h>

#include "../../oracle/oracle.h"
#include "../../tiflash_amd/host/planner.h"

using namespace tfa;

// ---------------------------------------------------------------- tiny test harness
static int g_failures = 0;
static std::string g_current;
#define EXPECT(cond)                                                                                     \
    do {                                                                                                 \
        if (!(cond)) {                                                                                   \
            ++g_failures;                                                                                \
            fprintf(stderr, "  FAILED %s:%d [%s]: %s\n", __FILE__, __LINE__, g_current.c_str(), #cond); \
        }                                                                                                \
    } while (0)

struct TestCase {
    const char *name;
    void (*fn)(Context &);
};
static std::vector<TestCase> &registry() {
    static std::vector<TestCase> r;
    return r;
}
struct Reg {
    Reg(const char *n, void (*f)(Context &)) { registry().push_back({n, f}); }
};
#define TEST(name)                                 \
    static void name(Context &ctx);                \
    static Reg reg_##name(#name, name);            \
    static void name(Context &ctx)

static std::string g_root;

// ---------------------------------------------------------------- minimal JSON (fixtures only)
struct Json {
    enum Kind { Null, Num, Str, Arr, Obj } kind = Null;
    double num = 0;
    std::string str;
    std::vector<Json> arr;
    std::vector<std::pair<std::string, Json>> obj;
    const Json &operator[](const std::string &k) const {
        for (const auto &kv : obj)
            if (kv.first == k) return kv.second;
        throw std::runtime_error("json key " + k);
    }
    const Json &operator[](size_t i) const { return arr.at(i); }
    size_t size() const { return kind == Arr ? arr.size() : obj.size(); }
};

struct JsonParser {
    const std::string &s;
    size_t i = 0;
    void ws() {
        while (i < s.size() && isspace((unsigned char)s[i])) ++i;
    }
    Json parse() {
        ws();
        Json j;
        if (s[i] == '{') {
            j.kind = Json::Obj;
            ++i;
            ws();
            if (s[i] == '}') {
                ++i;
                return j;
            }
            for (;;) {
                ws();
                std::string k = parse().str;
                ws();
                ++i; // ':'
                j.obj.push_back({k, parse()});
                ws();
                if (s[i++] == '}') return j;
            }
        }
        if (s[i] == '[') {
            j.kind = Json::Arr;
            ++i;
            ws();
            if (s[i] == ']') {
                ++i;
                return j;
            }
            for (;;) {
                j.arr.push_back(parse());
                ws();
                if (s[i++] == ']') return j;
            }
        }
        if (s[i] == '"') {
            j.kind = Json::Str;
            ++i;
            while (s[i] != '"') j.str += s[i++];
            ++i;
            return j;
        }
        if (s.compare(i, 4, "null") == 0) {
            i += 4;
            return j;
        }
        if (s.compare(i, 4, "true") == 0 || s.compare(i, 5, "false") == 0) {
            j.kind = Json::Num;
            j.num = s[i] == 't';
            i += s[i] == 't' ? 4 : 5;
            return j;
        }
        j.kind = Json::Num;
        size_t end = i;
        while (end < s.size() && (isdigit((unsigned char)s[end]) || strchr("+-.eE", s[end]))) ++end;
        j.num = atof(s.substr(i, end - i).c_str());
        i = end;
        return j;
    }
};

static Json load_fixture() {
    std::ifstream f(g_root + "/tests/golden/reference_cases.json");
    std::stringstream ss;
    ss << f.rdbuf();
    std::string text = ss.str();
    JsonParser p{text};
    return p.parse();
}

// nullable Int64 column from a JSON array with nulls
static ColumnWithTypeAndName jsonColumn(Context &ctx, const Json &arr, const std::string &name, int type = TFG_INT64) {
    const size_t n = arr.size();
    std::vector<int64_t> v(n, 0);
    std::vector<uint8_t> nm(n, 0);
    for (size_t i = 0; i < n; ++i) {
        if (arr[i].kind == Json::Null) nm[i] = 1;
        else v[i] = (int64_t)arr[i].num;
    }
    DataType t;
    t.type = type;
    t.nullable = true;
    const size_t w = t.width();
    std::vector<uint8_t> bytes(n * w);
    for (size_t i = 0; i < n; ++i) memcpy(bytes.data() + i * w, &v[i], w); // little-endian narrowing
    ColumnPtr c = makeColumn(ctx, t, bytes.data(), n, nm.data());
    return {c, c->type, name};
}

// values of a column as optional int64 (NULL -> "N") for multiset comparisons
static std::vector<std::string> cellStrings(Context &ctx, const IColumn &c) {
    std::vector<std::string> out(c.rows);
    std::vector<uint8_t> b = toHostBytes(ctx, c), nm = toHostNullMap(ctx, c);
    const size_t w = c.type.width();
    for (size_t i = 0; i < c.rows; ++i) {
        if (nm[i]) {
            out[i] = "N";
            continue;
        }
        int64_t v = 0;
        memcpy(&v, b.data() + i * w, w);
        if (w < 8 && c.type.type >= TFG_INT8 && c.type.type <= TFG_INT64) v = (v << (64 - 8 * w)) >> (64 - 8 * w);
        out[i] = std::to_string(v);
    }
    return out;
}

static std::vector<std::string> jsonStrings(const Json &arr) {
    std::vector<std::string> out;
    for (size_t i = 0; i < arr.size(); ++i)
        out.push_back(arr[i].kind == Json::Null ? "N" : std::to_string((int64_t)arr[i].num));
    return out;
}

// rows of a block as tuples, sorted (the reference compares results unordered)
static std::multiset<std::vector<std::string>> rowSet(Context &ctx, const Block &b) {
    std::vector<std::vector<std::string>> cols;
    for (const auto &c : b.getColumnsWithTypeAndName()) cols.push_back(cellStrings(ctx, *materialize(ctx, c.column)));
    std::multiset<std::vector<std::string>> rows;
    for (size_t r = 0; r < b.rows(); ++r) {
        std::vector<std::string> t;
        for (auto &c : cols) t.push_back(c[r]);
        rows.insert(t);
    }
    return rows;
}

static std::multiset<std::vector<std::string>> jsonRowSet(const Json &cols) {
    std::multiset<std::vector<std::string>> rows;
    if (cols.size() == 0) return rows;
    for (size_t r = 0; r < cols[0].size(); ++r) {
        std::vector<std::string> t;
        for (size_t c = 0; c < cols.size(); ++c)
            t.push_back(cols[c][r].kind == Json::Null ? "N" : std::to_string((int64_t)cols[c][r].num));
        rows.insert(t);
    }
    return rows;
}

// ================================================================ aggregation
// gtest_aggregation_executor.cpp:344-368 — GROUP BY each integer type with NULL keys
TEST(GroupByReferenceKnownAnswers) {
    Json fx = load_fixture();
    const Json &cases = fx["groupby"];
    for (size_t ci = 0; ci < cases.size(); ++ci) {
        const Json &c = cases[ci];
        g_current = "GroupBy " + c["name"].str;
        Block b{jsonColumn(ctx, c["column"], "k", (int)c["type"].num)};
        Aggregator::Params p;
        p.src_header = b;
        p.keys = {"k"};
        p.aggregates = {{"count", {}, "cnt"}};
        Aggregator agg(ctx, p);
        agg.executeOnBlock(b);
        Block res = agg.convertToBlock();
        std::vector<std::string> got = cellStrings(ctx, *res.getByName("k").column);
        std::vector<std::string> want = jsonStrings(c["expected"]);
        std::sort(got.begin(), got.end());
        std::sort(want.begin(), want.end());
        EXPECT(got == want);
        // counts add up to the input rows
        std::vector<uint64_t> cnt = toHost<uint64_t>(ctx, *res.getByName("cnt").column);
        uint64_t tot = 0;
        for (auto x : cnt) tot += x;
        EXPECT(tot == c["column"].size());
    }
}

// randomized: filter -> GROUP BY (sum Int64, sum nullable Float64, count) vs the CPU restatement
TEST(FilterGroupByMatchesOracle) {
    std::mt19937_64 rng(42);
    const size_t n = 300000;
    std::vector<int64_t> f(n), k(n), v(n);
    std::vector<double> d(n);
    std::vector<uint8_t> dn(n);
    for (size_t i = 0; i < n; ++i) {
        f[i] = rng() % 100;
        k[i] = (int64_t)(rng() % 20000) - 10000;
        v[i] = (int64_t)(rng() % 2000001) - 1000000;
        d[i] = (double)(rng() % (1 << 20)) / 256.0; // dyadic: exact in any order
        dn[i] = rng() % 7 == 0;
    }
    DataType i64, f64n;
    f64n.type = TFG_FLOAT64;
    f64n.nullable = true;
    Block b{{makeColumn(ctx, i64, f.data(), n), i64, "f"},
            {makeColumn(ctx, i64, k.data(), n), i64, "k"},
            {makeColumn(ctx, i64, v.data(), n), i64, "v"},
            {makeColumn(ctx, f64n, d.data(), n, dn.data()), f64n, "d"}};
    auto expr = std::make_shared<ExpressionActions>(ctx);
    expr->compare("f", TFG_LT, Field::Int64(70), "pred");
    Aggregator::Params p;
    p.src_header = b;
    p.keys = {"k"};
    p.aggregates = {{"sum", {"v"}, "sum_v"}, {"sum", {"d"}, "sum_d"}, {"count", {}, "cnt"}};
    // 1. through FilterBlockInputStream -> AggregatingBlockInputStream
    auto src = std::make_shared<BlocksListBlockInputStream>(std::vector<Block>{b});
    auto filt = std::make_shared<FilterBlockInputStream>(ctx, src, expr, "pred");
    AggregatingBlockInputStream aggs(ctx, filt, p);
    Block res = aggs.read();
    EXPECT(!aggs.read());
    // 2. the fused form
    Aggregator fused(ctx, p);
    fused.executeOnBlockFiltered(b, "f", TFG_LT, Field::Int64(70));
    Block res2 = fused.convertToBlock();
    // oracle
    std::vector<uint8_t> mask(n);
    for (size_t i = 0; i < n; ++i) mask[i] = f[i] < 70;
    int kinds[3] = {TFG_AGG_SUM, TFG_AGG_SUM, TFG_AGG_COUNT_ALL};
    int types[3] = {TFG_INT64, TFG_FLOAT64, 0};
    orc_agg *o = orc_agg_create(TFG_INT64, 3, kinds, types);
    const void *args[3] = {v.data(), d.data(), nullptr};
    const uint8_t *an[3] = {nullptr, dn.data(), nullptr};
    orc_agg_consume(o, k.data(), nullptr, args, an, mask.data(), n);
    const size_t g = orc_agg_size(o);
    std::vector<uint64_t> ok(g);
    std::vector<int64_t> os(g);
    std::vector<double> od(g);
    std::vector<uint64_t> oc(g);
    std::vector<uint8_t> okn(g), odn(g), on0(g), on2(g);
    void *outs[3] = {os.data(), od.data(), oc.data()};
    uint8_t *outn[3] = {on0.data(), odn.data(), on2.data()};
    orc_agg_result(o, ok.data(), okn.data(), outs, outn);
    orc_agg_destroy(o);
    std::map<int64_t, std::tuple<int64_t, double, uint8_t, uint64_t>> want;
    for (size_t i = 0; i < g; ++i) want[(int64_t)ok[i]] = {os[i], od[i], odn[i], oc[i]};
    for (const Block *r : {&res, &res2}) {
        g_current = r == &res ? "streams" : "fused";
        EXPECT(r->rows() == g);
        auto rk = toHost<int64_t>(ctx, *r->getByName("k").column);
        auto rs = toHost<int64_t>(ctx, *r->getByName("sum_v").column);
        auto rd = toHost<double>(ctx, *r->getByName("sum_d").column);
        auto rdn = toHostNullMap(ctx, *r->getByName("sum_d").column);
        auto rc = toHost<uint64_t>(ctx, *r->getByName("cnt").column);
        EXPECT(r->getByName("sum_d").column->type.nullable);
        size_t bad = 0;
        for (size_t i = 0; i < rk.size(); ++i) {
            auto it = want.find(rk[i]);
            if (it == want.end()) {
                ++bad;
                continue;
            }
            const auto &w = it->second;
            if (std::get<0>(w) != rs[i] || std::get<2>(w) != rdn[i] || std::get<3>(w) != rc[i]) ++bad;
            if (!rdn[i] && std::get<1>(w) != rd[i]) ++bad;
        }
        EXPECT(bad == 0);
    }
}

// two-phase aggregation: partial blocks of two "nodes" exchanged through HashPartitionWriter
// partitions, merged by a final Aggregator per partition (the MPP two-phase plan)
TEST(TwoPhaseAggregationThroughPartitions) {
    std::mt19937_64 rng(7);
    const size_t n = 100000;
    DataType i64;
    Aggregator::Params p;
    std::vector<std::vector<int64_t>> ks(2), vs(2);
    std::vector<Block> partial_parts[2];
    for (int node = 0; node < 2; ++node) {
        ks[node].resize(n);
        vs[node].resize(n);
        for (size_t i = 0; i < n; ++i) {
            ks[node][i] = rng() % 5000;
            vs[node][i] = rng() % 1000;
        }
        Block b{{makeColumn(ctx, i64, ks[node].data(), n), i64, "k"}, {makeColumn(ctx, i64, vs[node].data(), n), i64, "v"}};
        p.src_header = b;
        p.keys = {"k"};
        p.aggregates = {{"sum", {"v"}, "s"}, {"count", {}, "c"}};
        Aggregator partial(ctx, p);
        partial.executeOnBlock(b);
        Block pb = partial.convertToBlock(false);
        std::vector<Block> parts(3);
        HashPartitionWriter w(ctx, {0}, 3, [&](uint32_t part, Block &&blk) { parts[part] = std::move(blk); });
        w.write(pb);
        w.flush();
        partial_parts[node] = parts;
    }
    std::map<int64_t, std::pair<int64_t, uint64_t>> want;
    for (int node = 0; node < 2; ++node)
        for (size_t i = 0; i < n; ++i) {
            want[ks[node][i]].first += vs[node][i];
            want[ks[node][i]].second += 1;
        }
    size_t groups = 0, bad = 0;
    std::set<int64_t> seen;
    for (int part = 0; part < 3; ++part) {
        Block header = partial_parts[0][part];
        Aggregator::Params fp = p;
        Aggregator final_agg(ctx, fp);
        for (int node = 0; node < 2; ++node) final_agg.mergeOnBlock(partial_parts[node][part]);
        Block r = final_agg.convertToBlock();
        auto rk = toHost<int64_t>(ctx, *r.getByName("k").column);
        auto rs = toHost<int64_t>(ctx, *r.getByName("s").column);
        auto rc = toHost<uint64_t>(ctx, *r.getByName("c").column);
        groups += rk.size();
        for (size_t i = 0; i < rk.size(); ++i) {
            if (!seen.insert(rk[i]).second) ++bad; // a key lives in exactly one partition
            if (want[rk[i]] != std::make_pair(rs[i], rc[i])) ++bad;
        }
    }
    EXPECT(groups == want.size());
    EXPECT(bad == 0);
}

// ================================================================ join
// gtest_join_executor.cpp:114-200 — SimpleJoin inner/left/semi/anti, keys a and b, with NULLs
TEST(SimpleJoinReferenceKnownAnswers) {
    Json fx = load_fixture();
    const Json &cases = fx["join"];
    for (size_t ci = 0; ci < cases.size(); ++ci) {
        const Json &c = cases[ci];
        g_current = c["name"].str;
        const std::string kind = c["kind"].str;
        JoinKind jk = kind == "inner" ? JoinKind::Inner : kind == "left" ? JoinKind::Left
                    : kind == "semi"  ? JoinKind::Semi : JoinKind::Anti;
        const std::string key = c["key"].str;
        Block probe{jsonColumn(ctx, c["probe"]["a"], "l.a"), jsonColumn(ctx, c["probe"]["b"], "l.b")};
        Block build{jsonColumn(ctx, c["build"]["a"], "r.a"), jsonColumn(ctx, c["build"]["b"], "r.b")};
        Join join(ctx, jk, "l." + key, "r." + key);
        join.initBuild(build);
        join.insertFromBlock(build);
        join.finishOneBuild();
        Block out = join.joinBlock(probe);
        EXPECT(rowSet(ctx, out) == jsonRowSet(c["expected_columns"]));
    }
}

// randomized multi-block build with duplicate keys and NULLs vs the CPU restatement
TEST(JoinMatchesOracle) {
    std::mt19937_64 rng(3);
    const size_t nb = 50000, np = 200000;
    std::vector<int64_t> bk(nb), bp(nb), pk(np);
    std::vector<uint8_t> bn(nb), pn(np);
    for (size_t i = 0; i < nb; ++i) {
        bk[i] = rng() % 40000;
        bp[i] = (int64_t)i * 10;
        bn[i] = rng() % 50 == 0;
    }
    for (size_t i = 0; i < np; ++i) {
        pk[i] = rng() % 60000;
        pn[i] = rng() % 50 == 0;
    }
    DataType i64n;
    i64n.nullable = true;
    DataType i64;
    for (JoinKind jk : {JoinKind::Inner, JoinKind::Left, JoinKind::Semi, JoinKind::Anti}) {
        g_current = "kind " + std::to_string((int)jk);
        Join join(ctx, jk, "pk", "bk", nb);
        const size_t half = nb / 2;
        for (size_t part = 0; part < 2; ++part) {
            const size_t o = part * half, m = part ? nb - half : half;
            Block b{{makeColumn(ctx, i64n, bk.data() + o, m, bn.data() + o), i64n, "bk"},
                    {makeColumn(ctx, i64, bp.data() + o, m), i64, "bpay"}};
            join.insertFromBlock(b);
        }
        join.finishOneBuild();
        Block probe{{makeColumn(ctx, i64n, pk.data(), np, pn.data()), i64n, "pk"}};
        Block out = join.joinBlock(probe);
        // oracle pairs -> (probe key, build payload) multiset
        orc_join *oj = orc_join_create(TFG_INT64);
        orc_join_build(oj, bk.data(), bn.data(), nb);
        std::vector<uint32_t> op(np * 4), ob(np * 4);
        const size_t m = orc_join_probe(oj, (int)jk, pk.data(), pn.data(), np, op.data(), ob.data(), op.size());
        orc_join_destroy(oj);
        std::multiset<std::pair<std::string, std::string>> want, got;
        for (size_t i = 0; i < m; ++i) {
            const std::string kstr = pn[op[i]] ? "N" : std::to_string(pk[op[i]]);
            std::string bstr = "-";
            if (jk == JoinKind::Inner || jk == JoinKind::Left) bstr = ob[i] == 0xFFFFFFFFu ? "N" : std::to_string(bp[ob[i]]);
            want.insert({kstr, bstr});
        }
        auto gk = cellStrings(ctx, *out.getByName("pk").column);
        std::vector<std::string> gb(gk.size(), "-");
        if (jk == JoinKind::Inner || jk == JoinKind::Left) gb = cellStrings(ctx, *out.getByName("bpay").column);
        for (size_t i = 0; i < gk.size(); ++i) got.insert({gk[i], gb[i]});
        EXPECT(got == want);
    }
}

// ================================================================ filter
// gtest_filter_executor.cpp:74-285 style: predicates over nullable columns, all-false / all-true
TEST(FilterTransformActionSemantics) {
    DataType i64n;
    i64n.nullable = true;
    std::vector<int64_t> a = {1, 2, 3, 4, 5, 6};
    std::vector<uint8_t> an = {0, 0, 1, 0, 0, 0};
    std::vector<std::string> s = {"a", "bb", "", "dddd", "e", "ffffff"};
    Block header{{nullptr, i64n, "a"}, {nullptr, DataType{DataType::TYPE_STRING}, "s"}};
    auto make = [&]() {
        return Block{{makeColumn(ctx, i64n, a.data(), a.size(), an.data()), i64n, "a"},
                     {makeStringColumn(ctx, s), DataType{DataType::TYPE_STRING}, "s"}};
    };
    {
        g_current = "a >= 2";
        auto e = std::make_shared<ExpressionActions>(ctx);
        e->compare("a", TFG_GE, Field::Int64(2), "f");
        FilterTransformAction act(ctx, header, e, "f");
        Block b = make();
        FilterPtr fp;
        EXPECT(act.transform(b, fp, false));
        EXPECT(b.rows() == 4); // 2, 4, 5, 6 (the NULL row drops)
        auto av = toHost<int64_t>(ctx, *b.getByName("a").column);
        EXPECT((av == std::vector<int64_t>{2, 4, 5, 6}));
        auto sv = toHostStrings(ctx, *b.getByName("s").column);
        EXPECT((sv == std::vector<std::string>{"bb", "dddd", "e", "ffffff"}));
        EXPECT(b.getByName("f").column->isColumnConst());
    }
    {
        g_current = "all filtered";
        auto e = std::make_shared<ExpressionActions>(ctx);
        e->compare("a", TFG_GT, Field::Int64(100), "f");
        FilterTransformAction act(ctx, header, e, "f");
        Block b = make();
        FilterPtr fp;
        EXPECT(!act.transform(b, fp, false));
    }
    {
        g_current = "all pass";
        auto e = std::make_shared<ExpressionActions>(ctx);
        e->compare("a", TFG_LT, Field::Float64(100.5), "f");
        e->logical(TFG_NOT, "f", "", "nf");
        e->logical(TFG_OR, "nf", "f", "f2"); // NULL row: f = 0, not f = 1 -> passes
        FilterTransformAction act(ctx, header, e, "f2");
        Block b = make();
        FilterPtr fp;
        EXPECT(act.transform(b, fp, false));
        EXPECT(b.rows() == 6);
        EXPECT(b.getByName("f2").column->isColumnConst());
    }
    {
        g_current = "return_filter";
        auto e = std::make_shared<ExpressionActions>(ctx);
        e->compare("a", TFG_EQ, Field::Int64(4), "f");
        FilterTransformAction act(ctx, header, e, "f");
        Block b = make();
        FilterPtr fp;
        EXPECT(act.transform(b, fp, true));
        EXPECT(fp && (toHost<uint8_t>(ctx, *fp) == std::vector<uint8_t>{0, 0, 0, 1, 0, 0}));
    }
    {
        g_current = "illegal filter column type";
        auto e = std::make_shared<ExpressionActions>(ctx);
        e->arithmeticConst(TFG_PLUS, "a", Field::Int64(1), "f");
        FilterTransformAction act(ctx, header, e, "f");
        Block b = make();
        FilterPtr fp;
        int code = 0;
        try {
            act.transform(b, fp, false);
        } catch (const Exception &ex) {
            code = ex.code();
        }
        EXPECT(code == ErrorCodes::ILLEGAL_TYPE_OF_COLUMN_FOR_FILTER);
    }
    {
        g_current = "missing column";
        int code = 0;
        try {
            Block b = make();
            b.getByName("zz");
        } catch (const Exception &ex) {
            code = ex.code();
        }
        EXPECT(code == ErrorCodes::NOT_FOUND_COLUMN_IN_BLOCK);
    }
}

// random predicate columns vs the oracle's cmp + filterImpl, arithmetic with decimals
TEST(ExpressionsAndFilterMatchOracle) {
    std::mt19937_64 rng(11);
    const size_t n = 100003;
    std::vector<int64_t> x(n), y(n);
    std::vector<double> z(n);
    for (size_t i = 0; i < n; ++i) {
        x[i] = (int64_t)(rng() % 1000) - 500;
        y[i] = (int64_t)(rng() % 100000);
        z[i] = (double)(rng() % 1000) / 8.0;
    }
    DataType i64, f64, d64;
    f64.type = TFG_FLOAT64;
    d64.type = TFG_DECIMAL64;
    d64.scale = 2;
    Block b{{makeColumn(ctx, i64, x.data(), n), i64, "x"},
            {makeColumn(ctx, d64, y.data(), n), d64, "price"},
            {makeColumn(ctx, f64, z.data(), n), f64, "z"}};
    auto e = std::make_shared<ExpressionActions>(ctx);
    e->compare("x", TFG_LE, Field::Int64(100), "c1");
    e->compare("z", TFG_GT, Field::Float64(20.0), "c2");
    e->logical(TFG_AND, "c1", "c2", "f");
    e->arithmeticConst(TFG_MULTIPLY, "price", Field::Decimal64(95, 2), "disc_price"); // price * 0.95
    FilterTransformAction act(ctx, b.cloneEmpty(), e, "f");
    FilterPtr fp;
    EXPECT(act.transform(b, fp, false));
    std::vector<int64_t> wx;
    std::vector<__int128> wp;
    for (size_t i = 0; i < n; ++i)
        if (x[i] <= 100 && z[i] > 20.0) {
            wx.push_back(x[i]);
            wp.push_back((__int128)y[i] * 95);
        }
    EXPECT(b.rows() == wx.size());
    EXPECT(toHost<int64_t>(ctx, *b.getByName("x").column) == wx);
    const IColumn &dp = *b.getByName("disc_price").column;
    EXPECT(dp.type.type == TFG_DECIMAL128 && dp.type.scale == 4);
    auto gp = toHost<__int128>(ctx, dp);
    EXPECT(gp == wp);
}

// ================================================================ exchange
// gtest_mpp_exchange_writer.cpp:663-718 — 64 blocks of keys 0..63, P = 4 -> 1024 rows each
TEST(HashPartitionWriterKnownAnswer) {
    Json fx = load_fixture();
    const Json &ex = fx["exchange"];
    const size_t block_rows = (size_t)ex["block_rows"].num, blocks = (size_t)ex["blocks"].num;
    const uint32_t parts = (uint32_t)ex["parts"].num;
    std::vector<int64_t> keys(block_rows);
    for (size_t i = 0; i < block_rows; ++i) keys[i] = (int64_t)i;
    DataType i64;
    std::vector<size_t> got(parts, 0);
    size_t sends = 0;
    HashPartitionWriter w(ctx, {0}, parts, [&](uint32_t p, Block &&b) {
        got[p] += b.rows();
        ++sends;
    });
    for (size_t bi = 0; bi < blocks; ++bi) {
        Block b;
        for (int c = 0; c < 10; ++c) b.insert({makeColumn(ctx, i64, keys.data(), block_rows), i64, "c" + std::to_string(c)});
        w.write(b);
    }
    w.flush();
    for (uint32_t p = 0; p < parts; ++p) EXPECT(got[p] == (size_t)ex["rows_per_part"].num);
    EXPECT(sends == parts); // 4096 rows < 8192 * P: one flush
}

// FineGrainedShuffleWriter: the reference's known answers (gtest_mpp_exchange_writer.cpp:391-450,
// 542-607, numbers in tests/golden/reference_cases.json "fine_grained"): blocks of ten Int64
// columns 0..rows-1 partitioned on column 0, P = 4, S = 8.
//  * testBatchWriteFineGrainedShuffle: 1024 rows < batch 4096 * 8 -> one packet per partition,
//    S chunks each (stream ids 0..7), every chunk 1024 / 32 rows;
//  * testFineGrainedShuffleWriter(V1): 64 blocks of 64 rows + 64 empty blocks, batch 108 ->
//    1024 rows per partition and 512 rows per stream id over all packets.
TEST(FineGrainedShuffleWriterKnownAnswers) {
    Json fx = load_fixture();
    const Json &fg = fx["fine_grained"];
    const uint32_t P = (uint32_t)fg["parts"].num, S = (uint32_t)fg["streams"].num;
    DataType i64;
    auto block_of = [&](size_t rows) {
        std::vector<int64_t> v(std::max<size_t>(rows, 1));
        for (size_t i = 0; i < rows; ++i) v[i] = (int64_t)i;
        Block b;
        for (int c = 0; c < 10; ++c) b.insert({makeColumn(ctx, i64, v.data(), rows), i64, "col" + std::to_string(c)});
        return b;
    };
    { // one batch
        g_current = "FineGrainedShuffleWriter one batch";
        const Json &c = fg["batch"];
        Block block = block_of((size_t)c["block_rows"].num);
        std::map<uint32_t, FineGrainedPacket> report;
        FineGrainedShuffleWriter w(ctx, {0}, P, S, (uint64_t)c["batch_size"].num, [&](uint32_t p, FineGrainedPacket &&pk) {
            EXPECT(report.count(p) == 0); // a single flush: one packet per partition
            report[p] = std::move(pk);
        });
        w.write(block);
        w.flush();
        EXPECT(report.size() == P);
        size_t chunks = 0;
        for (auto &kv : report) {
            EXPECT(kv.second.chunks.size() == S && kv.second.stream_ids.size() == S);
            for (size_t i = 0; i < kv.second.chunks.size(); ++i) {
                Block d = CHBlockChunkCodecV1::decode(ctx, block.cloneEmpty(), kv.second.chunks[i]);
                EXPECT(d.rows() == (size_t)c["rows_per_chunk"].num);
                EXPECT(kv.second.stream_ids[i] == i);
                ++chunks;
            }
        }
        EXPECT(chunks == (size_t)P * S);
    }
    { // many small blocks, empty ones among them
        g_current = "FineGrainedShuffleWriter many blocks";
        const Json &c = fg["blocks"];
        const size_t rows = (size_t)c["block_rows"].num, nblocks = (size_t)c["block_num"].num;
        std::vector<size_t> part_rows(P, 0), stream_rows(S, 0);
        size_t packets = 0;
        Block header = block_of(0).cloneEmpty();
        FineGrainedShuffleWriter w(ctx, {0}, P, S, (uint64_t)c["batch_size"].num, [&](uint32_t p, FineGrainedPacket &&pk) {
            ++packets;
            EXPECT(pk.chunks.size() == pk.stream_ids.size());
            for (size_t i = 0; i < pk.chunks.size(); ++i) {
                Block d = CHBlockChunkCodecV1::decode(ctx, header, pk.chunks[i]);
                part_rows[p] += d.rows();
                stream_rows[pk.stream_ids[i]] += d.rows();
                // every row of the chunk routes to (p, stream id) under the reference's selector
                std::vector<int64_t> k = toHost<int64_t>(ctx, *d.getByName("col0").column);
                for (int64_t x : k) {
                    const uint32_t h = orc_crc32c_u64(0xFFFFFFFFu, (uint64_t)x); // intHashCRC32: crc32q
                    EXPECT((uint32_t)(((uint64_t)h * P) >> 32) == p && h % S == pk.stream_ids[i]);
                }
            }
        });
        for (size_t i = 0; i < nblocks; ++i) {
            w.write(block_of(rows));
            w.write(block_of(0));
        }
        w.flush();
        for (uint32_t p = 0; p < P; ++p) EXPECT(part_rows[p] == (size_t)c["rows_per_part"].num);
        for (uint32_t s = 0; s < S; ++s) EXPECT(stream_rows[s] == (size_t)c["rows_per_stream"].num);
        EXPECT(packets % P == 0 && packets > P); // several flushes, P packets each
    }
}

// one-rank RCCL exchange (the N>1 path runs in the multi-GPU bench): identity
TEST(MPPExchangeSingleRank) {
    uint8_t id[128];
    check(tfg_comm_unique_id(id, sizeof(id)), "tfg_comm_unique_id");
    MPPExchange ex(ctx, 1, 0, id, sizeof(id));
    std::vector<int64_t> k = {5, 6, 7, 8};
    std::vector<uint8_t> kn = {0, 1, 0, 0};
    DataType i64n;
    i64n.nullable = true;
    Block b{{makeColumn(ctx, i64n, k.data(), 4, kn.data()), i64n, "k"}};
    Block r = ex.exchange({b});
    EXPECT(cellStrings(ctx, *r.getByName("k").column) == (std::vector<std::string>{"5", "N", "7", "8"}));
    // a block with a String column travels as a CHBlockChunkCodecV1 packet
    DataType str{DataType::TYPE_STRING};
    Block bs{{makeColumn(ctx, i64n, k.data(), 4, kn.data()), i64n, "k"},
             {makeStringColumn(ctx, {"a", "", std::string(70, 'q'), "k00000001"}), str, "s"}};
    Block rs = ex.exchange({bs});
    EXPECT(cellStrings(ctx, *rs.getByName("k").column) == (std::vector<std::string>{"5", "N", "7", "8"}));
    EXPECT(toHostStrings(ctx, *rs.getByName("s").column) ==
           (std::vector<std::string>{"a", "", std::string(70, 'q'), "k00000001"}));
    Block es = ex.exchange({bs.cloneEmpty()}); // nothing sent, nothing received
    EXPECT(es.rows() == 0 && es.columns() == 2);
    // the planes follow the schema: a Nullable(Int64) column that carries no null map on this
    // rank (no NULLs here) still sends a null plane, and arrives Nullable with no NULLs
    auto nomap = std::make_shared<IColumn>(*makeColumn(ctx, i64n, k.data(), 4));
    nomap->nullmap.reset();
    Block bn{{nomap, i64n, "k"}};
    Block rn = ex.exchange({bn});
    EXPECT(rn.getByName("k").type.nullable && rn.getByName("k").column->nullmap);
    EXPECT(cellStrings(ctx, *rn.getByName("k").column) == (std::vector<std::string>{"5", "6", "7", "8"}));
    // and a non-Nullable schema never sends one
    DataType i64;
    Block bp{{makeColumn(ctx, i64, k.data(), 4), i64, "k"}};
    Block rp = ex.exchange({bp});
    EXPECT(!rp.getByName("k").type.nullable && !rp.getByName("k").column->nullmap);
}

// CHBlockChunkCodecV1 / CHBlockChunkCodec round trips through device packets (the reference's
// gtest_block_chunk_codec.cpp: encode nothing for an empty block, rows preserved, decode with
// the header's names; ExchangeReceiver decoding what HashPartitionWriter's sink encoded)
TEST(ChunkCodecRoundTrip) {
    std::vector<int64_t> k = {1, -2, 3, 1ll << 40, 5};
    std::vector<int32_t> x = {7, 0, 9, 10, 11};
    std::vector<uint8_t> xn = {0, 1, 0, 0, 1};
    std::vector<int64_t> d = {12345, -1, 0, 99, 100}; // Decimal(18,2)
    DataType i64, i32, dec, str;
    i32.type = TFG_INT32;
    str.type = DataType::TYPE_STRING;
    dec.type = TFG_DECIMAL64;
    dec.scale = 2;
    Block b{{makeColumn(ctx, i64, k.data(), 5), i64, "k"},
            {makeColumn(ctx, i32, x.data(), 5, xn.data()), i32, "x"},
            {makeColumn(ctx, dec, d.data(), 5), dec, "d"},
            {makeStringColumn(ctx, {"", "ab", std::string(300, 'z'), "\xff", "k00000001"}), str, "s"}};
    Block header = b.cloneEmpty();
    CHBlockChunkCodecV1 codec(ctx, header);
    EXPECT(codec.encode(header).empty()); // no rows: nothing encoded
    DevicePacket p = codec.encode(std::vector<Block>{b, b});
    EXPECT(codec.encoded_rows == 10);
    Block r = CHBlockChunkCodecV1::decode(ctx, header, p);
    EXPECT(r.rows() == 10 && r.columns() == 4);
    EXPECT(toHost<int64_t>(ctx, *r.getByName("k").column)[8] == (1ll << 40));
    EXPECT(cellStrings(ctx, *r.getByName("x").column)[6] == "N");
    EXPECT(r.getByName("d").column->type.scale == 2);
    EXPECT(toHost<int64_t>(ctx, *r.getByName("d").column)[5] == 12345);
    auto s = toHostStrings(ctx, *r.getByName("s").column);
    EXPECT(s[7] == std::string(300, 'z') && s[5].empty() && s[9] == "k00000001");
    CHBlockChunkCodec legacy(ctx, header);
    Block r2 = legacy.decode(legacy.encode(b));
    EXPECT(toHostStrings(ctx, *r2.getByName("s").column) == toHostStrings(ctx, *b.getByName("s").column));
    // ExchangeSender -> packets -> ExchangeReceiver (the exchange partitions fixed-width columns)
    Block bn = b;
    bn.erase(3);
    Block hn = bn.cloneEmpty();
    CHBlockChunkCodecV1 sender(ctx, hn);
    size_t rows = 0;
    HashPartitionWriter w(ctx, {0}, 3, [&](uint32_t, Block &&part) {
        DevicePacket pk = sender.encode(part);
        Block back = CHBlockChunkCodecV1::decode(ctx, hn, pk);
        rows += back ? back.rows() : 0;
    });
    w.write(bn);
    w.flush();
    EXPECT(rows == 5);
}

// Join with other conditions: the reference's SemiJoin known answers for `t.a = s.a and
// t.c < s.c` (gtest_join_executor.cpp:4400-4470: semi / anti / left-outer-semi /
// anti-left-outer-semi), and INNER / LEFT with the condition against a nested-loop restatement
// of Join::handleOtherConditions (NULL condition = no match).
static ColumnPtr i32col(Context &ctx, const std::vector<std::optional<int32_t>> &v) {
    std::vector<int32_t> x(v.size());
    std::vector<uint8_t> nm(v.size());
    for (size_t i = 0; i < v.size(); ++i) {
        x[i] = v[i].value_or(0);
        nm[i] = !v[i].has_value();
    }
    DataType t;
    t.type = TFG_INT32;
    return makeColumn(ctx, t, x.data(), v.size(), nm.data());
}

TEST(JoinOtherConditionKnownAnswers) {
    using V = std::vector<std::optional<int32_t>>;
    struct Case {
        V la, lc, ra, rc;
        std::vector<int> res;
    };
    const std::optional<int32_t> N;
    const std::vector<Case> cases = {
        {{1, 2, 3, 4, 5}, {1, 1, 1, 1, 1}, {1, 2, 3, 4, 5}, {2, 2, 2, 2, 2}, {1, 1, 1, 1, 1}},
        {{1, 2, 3, 4, 5}, {1, 1, 1, 1, 1}, {6, 7, 8, 9, 10}, {2, 2, 2, 2, 2}, {0, 0, 0, 0, 0}},
        {{1, 2, 3, 4, 5}, {1, 1, 1, 1, 1}, {}, {}, {0, 0, 0, 0, 0}},
        {{1, 1, 2, 2}, {1, N, 2, N}, {1, 1, 1, 2, 2, 2}, {N, 1, 2, 2, N, 3}, {1, 0, 1, 0}},
    };
    DataType i32;
    i32.type = TFG_INT32;
    for (const Case &cs : cases) {
        for (JoinKind kind : {JoinKind::Semi, JoinKind::Anti, JoinKind::LeftOuterSemi, JoinKind::AntiLeftOuterSemi}) {
            Block left{{i32col(ctx, cs.la), i32, "a"}, {i32col(ctx, cs.lc), i32, "c"}};
            Block right{{i32col(ctx, cs.ra), i32, "s_a"}, {i32col(ctx, cs.rc), i32, "s_c"}};
            Join j(ctx, kind, "a", "s_a");
            auto cond = std::make_shared<ExpressionActions>(ctx);
            cond->compareColumns("c", TFG_LT, "s_c", "other_cond");
            j.setOtherCondition(cond, "other_cond");
            j.insertFromBlock(right);
            j.finishOneBuild();
            Block r = j.joinBlock(left);
            std::vector<std::string> want_a;
            std::vector<std::string> want_match;
            for (size_t i = 0; i < cs.la.size(); ++i) {
                const bool m = cs.res[i] == 1;
                if (kind == JoinKind::Semi && m) want_a.push_back(std::to_string(*cs.la[i]));
                if (kind == JoinKind::Anti && !m) want_a.push_back(std::to_string(*cs.la[i]));
                if (kind == JoinKind::LeftOuterSemi) want_match.push_back(m ? "1" : "0");
                if (kind == JoinKind::AntiLeftOuterSemi) want_match.push_back(m ? "0" : "1");
            }
            if (kind == JoinKind::Semi || kind == JoinKind::Anti) {
                std::vector<std::string> got = cellStrings(ctx, *r.getByName("a").column);
                std::sort(got.begin(), got.end());
                std::sort(want_a.begin(), want_a.end());
                EXPECT(got == want_a);
            } else {
                EXPECT(r.rows() == cs.la.size());
                EXPECT(cellStrings(ctx, *r.getByName("match_helper").column) == want_match);
            }
        }
    }
}

TEST(JoinOtherConditionMatchesNestedLoop) {
    std::mt19937_64 rng(9);
    const size_t np = 300, nb = 120;
    std::vector<std::optional<int32_t>> pa(np), pc(np), ba(nb), bc(nb);
    for (auto &x : pa) x = (int32_t)(rng() % 25);
    for (auto &x : pc) x = rng() % 5 == 0 ? std::optional<int32_t>() : std::optional<int32_t>((int32_t)(rng() % 50));
    for (auto &x : ba) x = (int32_t)(rng() % 25);
    for (auto &x : bc) x = rng() % 5 == 0 ? std::optional<int32_t>() : std::optional<int32_t>((int32_t)(rng() % 50));
    pa[3] = std::nullopt; // a NULL probe key: never matched (LEFT keeps it with a NULL build side)
    DataType i32;
    i32.type = TFG_INT32;
    for (JoinKind kind : {JoinKind::Inner, JoinKind::Left}) {
        Block left{{i32col(ctx, pa), i32, "a"}, {i32col(ctx, pc), i32, "c"}};
        Block right{{i32col(ctx, ba), i32, "s_a"}, {i32col(ctx, bc), i32, "s_c"}};
        Join j(ctx, kind, "a", "s_a");
        auto cond = std::make_shared<ExpressionActions>(ctx);
        cond->compareColumns("c", TFG_LT, "s_c", "other_cond");
        j.setOtherCondition(cond, "other_cond");
        j.insertFromBlock(right);
        j.finishOneBuild();
        Block r = j.joinBlock(left);
        auto str = [](const std::optional<int32_t> &x) { return x ? std::to_string(*x) : std::string("N"); };
        std::multiset<std::vector<std::string>> want, got;
        for (size_t i = 0; i < np; ++i) {
            bool any = false;
            for (size_t b = 0; b < nb; ++b)
                if (pa[i] && ba[b] && *pa[i] == *ba[b] && pc[i] && bc[b] && *pc[i] < *bc[b]) {
                    want.insert({str(pa[i]), str(pc[i]), str(ba[b]), str(bc[b])});
                    any = true;
                }
            if (!any && kind == JoinKind::Left) want.insert({str(pa[i]), str(pc[i]), "N", "N"});
        }
        auto ca = cellStrings(ctx, *materialize(ctx, r.getByName("a").column));
        auto cc = cellStrings(ctx, *materialize(ctx, r.getByName("c").column));
        auto sa = cellStrings(ctx, *materialize(ctx, r.getByName("s_a").column));
        auto sc = cellStrings(ctx, *materialize(ctx, r.getByName("s_c").column));
        for (size_t i = 0; i < r.rows(); ++i) got.insert({ca[i], cc[i], sa[i], sc[i]});
        EXPECT(got == want);
    }
}

// General join keys (§8 f2, chooseJoinMapMethod keys128 / key_strbinpadding / serialized,
// JoinHashMap.cpp:33-116): two key columns (Int32, Nullable Int64) and one String key under the
// binary and the padding collator (strings longer than 16 bytes, trailing spaces, empty), each
// kind against a nested loop over the same rows.  A NULL in any key column never matches.
TEST(JoinGeneralKeysMatchNestedLoop) {
    std::mt19937_64 rng(21);
    const size_t np = 400, nb = 150;
    DataType i32, i64n, str{DataType::TYPE_STRING}, u8;
    i32.type = TFG_INT32;
    i64n.type = TFG_INT64;
    i64n.nullable = true;
    u8.type = TFG_UINT8;
    std::vector<std::string> words = {"", "a", "a ", "a  ", "b", "k00000001", "k00000001 ",
                                      "a fairly long join key over 16 bytes", "a fairly long join key over 16 bytez",
                                      " a", "z"};
    for (int collator : {-1 /* two fixed keys */, (int)TFG_COLLATOR_BINARY, (int)TFG_COLLATOR_BIN_PADDING}) {
        const bool fixed = collator < 0;
        std::vector<int32_t> pa(np), ba(nb);
        std::vector<int64_t> pb(np), bb(nb);
        std::vector<uint8_t> pbn(np), bbn(nb), ptag(np), btag(nb);
        std::vector<std::string> ps(np), bs(nb);
        for (size_t i = 0; i < np; ++i) {
            pa[i] = (int32_t)(rng() % 6);
            pb[i] = (int64_t)(rng() % 4) - 2;
            pbn[i] = rng() % 10 == 0;
            ps[i] = words[rng() % words.size()];
            ptag[i] = (uint8_t)(i % 251);
        }
        for (size_t i = 0; i < nb; ++i) {
            ba[i] = (int32_t)(rng() % 6);
            bb[i] = (int64_t)(rng() % 4) - 2;
            bbn[i] = rng() % 10 == 0;
            bs[i] = words[rng() % words.size()];
            btag[i] = (uint8_t)(i % 251);
        }
        auto trim = [&](std::string s) {
            if (collator == TFG_COLLATOR_BIN_PADDING)
                while (!s.empty() && s.back() == ' ') s.pop_back();
            return s;
        };
        auto eq = [&](size_t i, size_t b) {
            if (fixed) return !pbn[i] && !bbn[b] && pa[i] == ba[b] && pb[i] == bb[b];
            return trim(ps[i]) == trim(bs[b]);
        };
        for (JoinKind kind : {JoinKind::Inner, JoinKind::Left, JoinKind::Semi, JoinKind::Anti}) {
            Block left, right;
            if (fixed) {
                left = Block{{makeColumn(ctx, i32, pa.data(), np), i32, "a"},
                             {makeColumn(ctx, i64n, pb.data(), np, pbn.data()), i64n, "b"},
                             {makeColumn(ctx, u8, ptag.data(), np), u8, "ptag"}};
                right = Block{{makeColumn(ctx, i32, ba.data(), nb), i32, "s_a"},
                              {makeColumn(ctx, i64n, bb.data(), nb, bbn.data()), i64n, "s_b"},
                              {makeColumn(ctx, u8, btag.data(), nb), u8, "btag"}};
            } else {
                left = Block{{makeStringColumn(ctx, ps), str, "s"}, {makeColumn(ctx, u8, ptag.data(), np), u8, "ptag"}};
                right = Block{{makeStringColumn(ctx, bs), str, "s_s"},
                              {makeColumn(ctx, u8, btag.data(), nb), u8, "btag"}};
            }
            std::unique_ptr<Join> j;
            if (fixed)
                j = std::make_unique<Join>(ctx, kind, std::vector<std::string>{"a", "b"},
                                           std::vector<std::string>{"s_a", "s_b"});
            else
                j = std::make_unique<Join>(ctx, kind, std::vector<std::string>{"s"}, std::vector<std::string>{"s_s"},
                                           0, std::vector<int>{collator});
            j->insertFromBlock(right);
            j->finishOneBuild();
            Block r = j->joinBlock(left);
            std::multiset<std::pair<std::string, std::string>> want, got;
            for (size_t i = 0; i < np; ++i) {
                bool any = false;
                for (size_t b = 0; b < nb; ++b)
                    if (eq(i, b)) {
                        any = true;
                        if (kind == JoinKind::Inner || kind == JoinKind::Left)
                            want.insert({std::to_string(ptag[i]) + "/" + std::to_string(i), std::to_string(btag[b])});
                    }
                if (!any && kind == JoinKind::Left) want.insert({std::to_string(ptag[i]) + "/" + std::to_string(i), "N"});
                if ((any && kind == JoinKind::Semi) || (!any && kind == JoinKind::Anti))
                    want.insert({std::to_string(ptag[i]) + "/" + std::to_string(i), ""});
            }
            // probe row identity: ptag plus the row's key text (rows are unique by construction
            // only through the tag and keys; compare (tag, keys) multisets instead of row ids)
            std::vector<std::string> tags = cellStrings(ctx, *materialize(ctx, r.getByName("ptag").column));
            std::vector<std::string> keys;
            if (fixed) {
                auto a = cellStrings(ctx, *materialize(ctx, r.getByName("a").column));
                auto b = cellStrings(ctx, *materialize(ctx, r.getByName("b").column));
                for (size_t i = 0; i < r.rows(); ++i) keys.push_back(a[i] + "," + b[i]);
            } else {
                keys = toHostStrings(ctx, *r.getByName("s").column);
            }
            std::vector<std::string> bt;
            if (kind == JoinKind::Inner || kind == JoinKind::Left)
                bt = cellStrings(ctx, *materialize(ctx, r.getByName("btag").column));
            for (size_t i = 0; i < r.rows(); ++i)
                got.insert({tags[i] + "|" + keys[i], bt.empty() ? "" : bt[i]});
            // expected in the same (tag | keys) form
            std::multiset<std::pair<std::string, std::string>> want2;
            for (const auto &w : want) {
                const size_t i = std::stoul(w.first.substr(w.first.find('/') + 1));
                const std::string k = fixed ? std::to_string(pa[i]) + "," + (pbn[i] ? std::string("N") : std::to_string(pb[i]))
                                            : ps[i];
                want2.insert({std::to_string(ptag[i]) + "|" + k, w.second});
            }
            EXPECT(got == want2);
        }
    }
}

// Aggregator with several fixed keys (keys128 / nullable_keys128) and with one String key
// (key_string under the padding collator): executeOnBlock, the fused filter, two-phase
// convertToBlock(false) -> mergeOnBlock, against std::map over the same rows.
TEST(AggregatorPackedKeysMatchMap) {
    std::mt19937_64 rng(31);
    const size_t n = 20000;
    DataType i32, i16n, i64, str{DataType::TYPE_STRING};
    i32.type = TFG_INT32;
    i16n.type = TFG_INT16;
    i16n.nullable = true;
    std::vector<int32_t> a(n);
    std::vector<int16_t> b(n);
    std::vector<uint8_t> bn(n);
    std::vector<int64_t> v(n), f(n);
    std::vector<std::string> s(n);
    // the last two are past key_string's 15 bytes: the String-key aggregator moves to serialized
    const std::vector<std::string> words = {"",  "x", "x ", "k00000001", "k00000001  ", "abcdefghijklmno", " y",
                                            "customer-name-000000000042", "customer-name-000000000042   "};
    for (size_t i = 0; i < n; ++i) {
        a[i] = (int32_t)(rng() % 50) - 25;
        b[i] = (int16_t)(rng() % 7);
        bn[i] = rng() % 9 == 0;
        v[i] = (int64_t)(rng() % 1000) - 500;
        f[i] = (int64_t)(rng() % 10);
        s[i] = words[rng() % words.size()];
    }
    Block blk{{makeColumn(ctx, i32, a.data(), n), i32, "a"},
              {makeColumn(ctx, i16n, b.data(), n, bn.data()), i16n, "b"},
              {makeStringColumn(ctx, s), str, "s"},
              {makeColumn(ctx, i64, v.data(), n), i64, "v"},
              {makeColumn(ctx, i64, f.data(), n), i64, "f"}};
    for (int mode = 0; mode < 3; ++mode) { // 0: (a, b) keys, 1: String key s, 2: (a, s) serialized
        Aggregator::Params p;
        p.keys = mode == 0   ? std::vector<std::string>{"a", "b"}
                 : mode == 1 ? std::vector<std::string>{"s"}
                             : std::vector<std::string>{"a", "s"};
        if (mode == 1) p.collators = {TFG_COLLATOR_BIN_PADDING};
        if (mode == 2) p.collators = {TFG_COLLATOR_NONE, TFG_COLLATOR_BIN_PADDING};
        p.aggregates = {{"sum", {"v"}, "sum_v"}, {"count", {}, "cnt"}};
        p.src_header = blk.cloneEmpty();
        auto keyOf = [&](size_t i) {
            if (mode == 0) return std::to_string(a[i]) + "," + (bn[i] ? std::string("N") : std::to_string(b[i]));
            std::string t = s[i];
            while (!t.empty() && t.back() == ' ') t.pop_back();
            return mode == 2 ? std::to_string(a[i]) + "," + t : t;
        };
        for (int filtered = 0; filtered < 2; ++filtered) {
            std::map<std::string, std::pair<int64_t, uint64_t>> want;
            for (size_t i = 0; i < n; ++i) {
                if (filtered && !(f[i] < 7)) continue;
                auto &w = want[keyOf(i)];
                w.first += v[i];
                w.second += 1;
            }
            // phase 1 over two halves (two partial aggregators), phase 2 merges their blocks
            Aggregator final_agg(ctx, p);
            for (int half = 0; half < 2; ++half) {
                Aggregator part(ctx, p);
                std::vector<uint32_t> rows;
                for (size_t i = half; i < n; i += 2) rows.push_back((uint32_t)i);
                DeviceBuffer perm(ctx, rows.size() * 4);
                check(tfg_upload(ctx.raw(), perm.data(), rows.data(), rows.size() * 4), "tfg_upload");
                Block hb;
                for (const auto &c : blk.getColumnsWithTypeAndName()) {
                    ColumnPtr g = gatherColumn(ctx, *c.column, (const uint32_t *)perm.data(), rows.size(), false);
                    hb.insert({g, g->type, c.name});
                }
                if (filtered)
                    part.executeOnBlockFiltered(hb, "f", TFG_LT, Field::Int64(7));
                else
                    part.executeOnBlock(hb);
                final_agg.mergeOnBlock(part.convertToBlock(false));
            }
            Block r = final_agg.convertToBlock(true);
            std::map<std::string, std::pair<int64_t, uint64_t>> got;
            std::vector<std::string> keys;
            if (mode == 0) {
                auto ka = cellStrings(ctx, *r.getByName("a").column);
                auto kb = cellStrings(ctx, *r.getByName("b").column);
                for (size_t i = 0; i < r.rows(); ++i) keys.push_back(ka[i] + "," + kb[i]);
            } else if (mode == 1) {
                keys = toHostStrings(ctx, *r.getByName("s").column);
            } else {
                auto ka = cellStrings(ctx, *r.getByName("a").column);
                auto ks = toHostStrings(ctx, *r.getByName("s").column);
                for (size_t i = 0; i < r.rows(); ++i) keys.push_back(ka[i] + "," + ks[i]);
            }
            auto sums = toHost<int64_t>(ctx, *r.getByName("sum_v").column);
            auto cnts = toHost<uint64_t>(ctx, *r.getByName("cnt").column);
            for (size_t i = 0; i < r.rows(); ++i) got[keys[i]] = {sums[i], cnts[i]};
            EXPECT(r.rows() == want.size());
            EXPECT(got == want);
        }
    }
}

// HashPartitionWriter over a block with String columns (partition keys: a String under the
// padding collator, then a Nullable Int64): the rows of every partition, in order, equal the
// oracle's weak hash -> fillSelector -> stable partition of the same rows.
TEST(HashPartitionStringColumnsMatchOracle) {
    std::mt19937_64 rng(41);
    const size_t n = 5000;
    const uint32_t P = 5;
    DataType i64n, str{DataType::TYPE_STRING};
    i64n.nullable = true;
    std::vector<std::string> s(n);
    std::vector<int64_t> k(n), tag(n);
    std::vector<uint8_t> kn(n), sn(n);
    for (size_t i = 0; i < n; ++i) {
        s[i] = "k" + std::to_string(rng() % 300) + std::string(rng() % 3, ' ');
        k[i] = (int64_t)(rng() % 40) - 20;
        kn[i] = rng() % 8 == 0;
        sn[i] = rng() % 11 == 0;
        tag[i] = (int64_t)i;
    }
    DataType str_n = str;
    str_n.nullable = true;
    Block blk{{makeStringColumn(ctx, s, sn.data()), str_n, "s"},
              {makeColumn(ctx, i64n, k.data(), n, kn.data()), i64n, "k"},
              {makeColumn(ctx, DataType{}, tag.data(), n), DataType{}, "tag"}};
    std::vector<Block> got(P);
    HashPartitionWriter w(ctx, {0, 1}, P, [&](uint32_t p, Block &&b) { got[p] = std::move(b); }, 1);
    w.setCollators({TFG_COLLATOR_BIN_PADDING, TFG_COLLATOR_NONE});
    w.write(blk);
    w.flush();
    // oracle: same hash chain over host copies
    std::string chars;
    std::vector<uint64_t> offs(n);
    for (size_t i = 0; i < n; ++i) {
        chars += s[i];
        chars.push_back('\0');
        offs[i] = chars.size();
    }
    std::vector<uint32_t> h(n, 0xFFFFFFFFu), sel(n), perm(n);
    std::vector<uint64_t> po(P + 1);
    orc_weak_hash_update_string((const uint8_t *)chars.data(), offs.data(), sn.data(), n, TFG_COLLATOR_BIN_PADDING,
                                h.data());
    orc_weak_hash_update(TFG_INT64, k.data(), kn.data(), n, h.data());
    orc_fill_selector(h.data(), n, P, 0, sel.data());
    orc_partition(sel.data(), n, P, perm.data(), po.data());
    (void)w;
    for (uint32_t p = 0; p < P; ++p) {
        std::vector<std::string> want_tag, want_s;
        for (uint64_t r = po[p]; r < po[p + 1]; ++r) {
            want_tag.push_back(std::to_string(perm[r]));
            want_s.push_back(sn[perm[r]] ? "N" : s[perm[r]]);
        }
        EXPECT(got[p].rows() == want_tag.size());
        if (!got[p].rows()) continue;
        EXPECT(cellStrings(ctx, *got[p].getByName("tag").column) == want_tag);
        auto gs = toHostStrings(ctx, *got[p].getByName("s").column);
        auto gn = toHostNullMap(ctx, *got[p].getByName("s").column);
        for (size_t i = 0; i < gs.size(); ++i)
            if (gn[i]) gs[i] = "N";
        EXPECT(gs == want_s);
    }
}

// AutoPassThroughHashAggContext: the reference's state machine driven by three key
// distributions (all-new keys -> PassThrough, few keys -> stays Init, half-known keys ->
// Selective); pass-through blocks + the hash map's block, merged as the second stage would,
// must equal a direct aggregation of the input.
TEST(AutoPassThroughHashAgg) {
    DataType i64, i32n;
    i32n.type = TFG_INT32;
    i32n.nullable = true;
    Aggregator::Params p;
    p.keys = {"k"};
    p.aggregates = {{"sum", {"v"}, "sum_v"}, {"count", {"v"}, "cnt_v"}, {"count", {}, "cnt"}};
    p.src_header = Block{{nullptr, i64, "k"}, {nullptr, i32n, "v"}};
    const size_t B = 8192;
    auto run = [&](int scenario, size_t blocks, size_t &pass_rows, std::set<int> &states) {
        AutoPassThroughHashAggContext apt(ctx, p, /*row_limit_unit=*/B);
        std::mt19937_64 rng(77 + scenario);
        std::map<int64_t, std::tuple<int64_t, uint64_t, uint64_t, bool>> want; // sum, cnt_v, cnt, any non-null
        std::vector<Block> out;
        int64_t next_new = 0;
        for (size_t bi = 0; bi < blocks; ++bi) {
            std::vector<int64_t> k(B);
            std::vector<int32_t> v(B);
            std::vector<uint8_t> vn(B);
            for (size_t i = 0; i < B; ++i) {
                if (scenario == 0) k[i] = next_new++;                            // every key new
                else if (scenario == 1) k[i] = (int64_t)(rng() % 1000);          // few keys
                else k[i] = bi < 9 || rng() % 2 ? (bi < 9 ? next_new++ : (int64_t)(rng() % 70000)) : 1000000 + next_new++;
                v[i] = (int32_t)(rng() % 1000) - 500;
                vn[i] = rng() % 7 == 0;
                auto &w = want[k[i]];
                if (!vn[i]) {
                    std::get<0>(w) += v[i];
                    std::get<1>(w) += 1;
                    std::get<3>(w) = true;
                }
                std::get<2>(w) += 1;
            }
            Block b{{makeColumn(ctx, i64, k.data(), B), i64, "k"}, {makeColumn(ctx, i32n, v.data(), B, vn.data()), i32n, "v"}};
            apt.onBlock(b);
            states.insert((int)apt.state());
            while (Block r = apt.tryGetDataInAdvance()) out.push_back(r);
        }
        if (Block h = apt.getDataFromHashTable()) out.push_back(h);
        pass_rows = apt.passThroughRows();
        std::map<int64_t, std::tuple<int64_t, uint64_t, uint64_t, bool>> got;
        for (const Block &b : out) {
            auto kk = toHost<int64_t>(ctx, *materialize(ctx, b.getByName("k").column));
            auto sc = b.getByName("sum_v").column;
            auto ss = toHost<int64_t>(ctx, *sc);
            auto sn = toHostNullMap(ctx, *sc);
            auto c1 = toHost<uint64_t>(ctx, *materialize(ctx, b.getByName("cnt_v").column));
            auto c2 = toHost<uint64_t>(ctx, *materialize(ctx, b.getByName("cnt").column));
            for (size_t i = 0; i < kk.size(); ++i) {
                auto &g = got[kk[i]];
                if (!sn[i]) {
                    std::get<0>(g) += ss[i];
                    std::get<3>(g) = true;
                }
                std::get<1>(g) += c1[i];
                std::get<2>(g) += c2[i];
            }
        }
        EXPECT(got == want);
    };
    size_t pass = 0;
    std::set<int> st;
    run(0, 30, pass, st);
    EXPECT(pass > 0 && st.count((int)AutoPassThroughHashAggContext::State::PassThrough));
    st.clear();
    run(1, 10, pass, st);
    EXPECT(pass == 0 && st == std::set<int>{(int)AutoPassThroughHashAggContext::State::Init});
    st.clear();
    run(2, 30, pass, st);
    EXPECT(pass > 0 && st.count((int)AutoPassThroughHashAggContext::State::Selective));
}

// The spill hand-off of auto pass-through (AutoPassThroughHashAggContext.cpp:86-104,
// Aggregator.cpp:79-92,1236-1243): once the map's revocable bytes pass the spill threshold it is
// marked for spill, forceState keeps every later block in PassThrough, and tryGetDataInAdvance
// hands the map's final block over first (once).  The merged output equals a host aggregation;
// the external trigger (AggregateContext::needSpill with try_mark) refuses an empty map.
TEST(AutoPassThroughSpillHandOff) {
    DataType i64;
    Aggregator::Params p;
    p.keys = {"k"};
    p.aggregates = {{"sum", {"v"}, "sum_v"}, {"count", {}, "cnt"}};
    p.src_header = Block{{nullptr, i64, "k"}, {nullptr, i64, "v"}};
    const size_t B = 4096;
    std::mt19937_64 rng(91);
    for (int external = 0; external < 2; ++external) {
        g_current = external ? "spill hand-off, external trigger" : "spill hand-off, threshold";
        // few keys (the map would stay in Init without a spill); threshold ~ 6K groups' bytes
        AutoPassThroughHashAggContext apt(ctx, p, /*row_limit_unit=*/B, 1, 5, external ? 0 : 200 * 1024);
        std::map<int64_t, std::pair<int64_t, uint64_t>> want, got;
        size_t pass_before = 0, marked_at = 0, map_rows = 0;
        bool handed = false, first_after_mark_is_map = false;
        for (size_t bi = 0; bi < 24; ++bi) {
            std::vector<int64_t> k(B), v(B);
            for (size_t i = 0; i < B; ++i) {
                k[i] = (int64_t)(rng() % 9000);
                v[i] = (int64_t)(rng() % 100);
                want[k[i]].first += v[i];
                want[k[i]].second += 1;
            }
            Block b{{makeColumn(ctx, i64, k.data(), B), i64, "k"}, {makeColumn(ctx, i64, v.data(), B), i64, "v"}};
            if (external && bi == 5) EXPECT(apt.tryMarkNeedSpill());
            const bool was_marked = apt.needSpill();
            pass_before = apt.passThroughRows();
            apt.onBlock(b);
            // forceState: the block passed through, the map took nothing (the state may read
            // Adjust afterwards: trySwitchBackAdjustState runs after the block, forceState
            // puts it back before the next one)
            if (was_marked) EXPECT(apt.passThroughRows() == pass_before + B);
            if (apt.needSpill() && !marked_at) marked_at = bi + 1;
            bool first = true;
            while (Block r = apt.tryGetDataInAdvance()) {
                if (apt.needSpill() && !handed) {
                    handed = true;
                    first_after_mark_is_map = first && r.rows() > 0 && r.rows() <= 9000;
                    map_rows = r.rows();
                }
                first = false;
                auto kk = toHost<int64_t>(ctx, *materialize(ctx, r.getByName("k").column));
                auto ss = toHost<int64_t>(ctx, *materialize(ctx, r.getByName("sum_v").column));
                auto cc = toHost<uint64_t>(ctx, *materialize(ctx, r.getByName("cnt").column));
                for (size_t i = 0; i < kk.size(); ++i) {
                    got[kk[i]].first += ss[i];
                    got[kk[i]].second += cc[i];
                }
            }
        }
        EXPECT(marked_at > 0 && marked_at < 24 && handed && first_after_mark_is_map && map_rows > 0);
        EXPECT(!apt.getDataFromHashTable()); // already handed over
        EXPECT(got == want);
        EXPECT(apt.passThroughRows() >= (24 - marked_at) * B);
    }
    { // the external trigger refuses an empty map (tryMarkNeedSpill: empty() -> false)
        AutoPassThroughHashAggContext apt(ctx, p, B);
        EXPECT(!apt.tryMarkNeedSpill() && !apt.needSpill());
    }
}

// Two GROUP BY keys (Int64, Nullable(Int32)) through the pass-through state machine: the first
// key alone collides constantly (1000 values), so a Selective-state lookup on it alone would call
// new tuples hits.  The lookup runs on the full tuple; tuples holding a NULL pass through.  Every
// output block carries both keys, and the merged result equals a host aggregation of the input.
TEST(AutoPassThroughHashAggTwoKeys) {
    DataType i64, i32n;
    i32n.type = TFG_INT32;
    i32n.nullable = true;
    Aggregator::Params p;
    p.keys = {"k1", "k2"};
    p.aggregates = {{"sum", {"v"}, "sum_v"}, {"count", {}, "cnt"}};
    p.src_header = Block{{nullptr, i64, "k1"}, {nullptr, i32n, "k2"}, {nullptr, i64, "v"}};
    const size_t B = 8192;
    AutoPassThroughHashAggContext apt(ctx, p, /*row_limit_unit=*/B);
    std::mt19937_64 rng(91);
    using Key = std::tuple<int64_t, int64_t>; // k2 = INT64_MIN stands for NULL
    std::map<Key, std::pair<int64_t, uint64_t>> want;
    std::vector<Block> out;
    std::set<int> states;
    int64_t next_new = 0;
    for (size_t bi = 0; bi < 30; ++bi) {
        std::vector<int64_t> k1(B), v(B);
        std::vector<int32_t> k2(B);
        std::vector<uint8_t> k2n(B);
        for (size_t i = 0; i < B; ++i) {
            const int64_t key = bi < 9 ? next_new++ : rng() % 2 ? (int64_t)(rng() % 70000) : 1000000 + next_new++;
            k1[i] = key % 1000;
            k2[i] = (int32_t)(key / 1000);
            k2n[i] = rng() % 50 == 0;
            v[i] = (int64_t)(rng() % 1000) - 500;
            auto &w = want[Key{k1[i], k2n[i] ? INT64_MIN : (int64_t)k2[i]}];
            w.first += v[i];
            w.second += 1;
        }
        Block b{{makeColumn(ctx, i64, k1.data(), B), i64, "k1"},
                {makeColumn(ctx, i32n, k2.data(), B, k2n.data()), i32n, "k2"},
                {makeColumn(ctx, i64, v.data(), B), i64, "v"}};
        apt.onBlock(b); // throws "Selective state grew the hash map" on a false hit
        states.insert((int)apt.state());
        while (Block r = apt.tryGetDataInAdvance()) out.push_back(r);
    }
    if (Block h = apt.getDataFromHashTable()) out.push_back(h);
    EXPECT(apt.passThroughRows() > 0 && states.count((int)AutoPassThroughHashAggContext::State::Selective));
    std::map<Key, std::pair<int64_t, uint64_t>> got;
    for (const Block &b : out) {
        EXPECT(b.has("k1") && b.has("k2"));
        auto a1 = toHost<int64_t>(ctx, *materialize(ctx, b.getByName("k1").column));
        auto a2c = materialize(ctx, b.getByName("k2").column);
        auto a2 = toHost<int32_t>(ctx, *a2c);
        auto a2n = toHostNullMap(ctx, *a2c);
        auto sv = toHost<int64_t>(ctx, *materialize(ctx, b.getByName("sum_v").column));
        auto c = toHost<uint64_t>(ctx, *materialize(ctx, b.getByName("cnt").column));
        for (size_t i = 0; i < a1.size(); ++i) {
            auto &g = got[Key{a1[i], a2n[i] ? INT64_MIN : (int64_t)a2[i]}];
            g.first += sv[i];
            g.second += c[i];
        }
    }
    EXPECT(got == want);
}

// Decimal precision (DataTypeDecimal(prec, scale)) through the operators: sum(Decimal(p, s)) ->
// Decimal(min(p + 22, 65), s) (SumDecimalInferer, Common/Decimal.h:156-163): Decimal(15,2) keeps an
// Int128 state, Decimal(18,2) and Decimal(38,4) a Decimal256 one (exact past Int128); and the
// packet header names the column's real precision, so the V1 packet of a Decimal(15,2) column is
// byte-identical to the oracle's (CodecUtils::checkDataTypeName on the receiver compares names).
static void add256(uint64_t *a, __int128 v) {
    const uint64_t x[4] = {(uint64_t)v, (uint64_t)((unsigned __int128)v >> 64), v < 0 ? ~0ull : 0ull, v < 0 ? ~0ull : 0ull};
    unsigned __int128 c = 0;
    for (int k = 0; k < 4; ++k) {
        c += (unsigned __int128)a[k] + x[k];
        a[k] = (uint64_t)c;
        c >>= 64;
    }
}

TEST(DecimalPrecisionSumAndCodec) {
    const size_t n = 50000;
    std::mt19937_64 rng(77);
    std::vector<int64_t> k(n), d15(n), d18(n);
    std::vector<__int128> d38(n);
    for (size_t i = 0; i < n; ++i) {
        k[i] = (int64_t)(rng() % 300);
        d15[i] = (int64_t)(rng() % 1999999999999999ull) - 999999999999999ll;
        d18[i] = (int64_t)(rng() % 1999999999999999999ull) - 999999999999999999ll;
        const __int128 hi = (__int128)((rng() % (1ull << 61)) + (1ull << 61)) * ((rng() % 5) ? 1 : -1);
        d38[i] = (hi << 64) + (__int128)rng();
    }
    DataType i64;
    DataType t15 = DataType::decimal(15, 2), t18 = DataType::decimal(18, 2), t38 = DataType::decimal(38, 4);
    EXPECT(t15.type == TFG_DECIMAL64 && t18.type == TFG_DECIMAL64 && t38.type == TFG_DECIMAL128);
    EXPECT(t15.getName() == "Decimal(15,2)" && t38.getName() == "Decimal(38,4)");
    EXPECT(!(t15 == t18));
    Block b{{makeColumn(ctx, i64, k.data(), n), i64, "k"},
            {makeColumn(ctx, t15, d15.data(), n), t15, "d15"},
            {makeColumn(ctx, t18, d18.data(), n), t18, "d18"},
            {makeColumn(ctx, t38, d38.data(), n), t38, "d38"}};
    Aggregator::Params p;
    p.src_header = b;
    p.keys = {"k"};
    p.aggregates = {{"sum", {"d15"}, "s15"}, {"sum", {"d18"}, "s18"}, {"sum", {"d38"}, "s38"}};
    Aggregator agg(ctx, p);
    agg.executeOnBlock(b);
    Block r = agg.convertToBlock();
    const IColumn &s15 = *r.getByName("s15").column, &s18 = *r.getByName("s18").column, &s38 = *r.getByName("s38").column;
    EXPECT(s15.type.type == TFG_DECIMAL128 && s15.type.getName() == "Decimal(37,2)");
    EXPECT(s18.type.type == TFG_DECIMAL256 && s18.type.getName() == "Decimal(40,2)" && s18.type.width() == 32);
    EXPECT(s38.type.type == TFG_DECIMAL256 && s38.type.getName() == "Decimal(60,4)");
    std::map<int64_t, std::vector<uint64_t>> want; // key -> 3 x 4 limbs
    for (size_t i = 0; i < n; ++i) {
        auto &w = want[k[i]];
        w.resize(12);
        add256(&w[0], d15[i]);
        add256(&w[4], d18[i]);
        add256(&w[8], d38[i]);
    }
    auto rk = toHost<int64_t>(ctx, *r.getByName("k").column);
    auto b15 = toHostBytes(ctx, s15), b18 = toHostBytes(ctx, s18), b38 = toHostBytes(ctx, s38);
    EXPECT(rk.size() == want.size());
    bool past128 = false;
    for (size_t g = 0; g < rk.size(); ++g) {
        const auto &w = want[rk[g]];
        __int128 v15;
        memcpy(&v15, b15.data() + 16 * g, 16);
        uint64_t lo15[4] = {0, 0, 0, 0};
        add256(lo15, v15);
        EXPECT(memcmp(lo15, &w[0], 32) == 0);
        EXPECT(memcmp(b18.data() + 32 * g, &w[4], 32) == 0);
        EXPECT(memcmp(b38.data() + 32 * g, &w[8], 32) == 0);
        past128 = past128 || (w[10] != 0 && w[10] != ~0ull) || ((w[9] >> 63) != (w[10] & 1));
    }
    EXPECT(past128); // some Decimal(38,4) sums leave Int128
    // codec: the Decimal(15,2) header and bytes equal the oracle's packet
    Block cb{{b.getByName("d15").column, t15, "d15"}};
    CHBlockChunkCodecV1 codec(ctx, cb.cloneEmpty());
    DevicePacket pk = codec.encode(cb);
    std::vector<uint8_t> got(pk.bytes);
    check(tfg_download(ctx.raw(), got.data(), pk.buf->data(), pk.bytes), "download");
    const char *names[1] = {"d15"}, *types[1] = {"Decimal(15,2)"};
    const void *data[1] = {d15.data()};
    const uint64_t *offs[1] = {nullptr};
    const uint8_t *nms[1] = {nullptr};
    const size_t want_bytes = orc_codec_encode(TFG_CODEC_V1, 1, names, types, data, offs, nms, (int64_t)n, 0, nullptr,
                                               nullptr, 0);
    std::vector<uint8_t> exp(want_bytes);
    orc_codec_encode(TFG_CODEC_V1, 1, names, types, data, offs, nms, (int64_t)n, 0, nullptr, exp.data(), exp.size());
    EXPECT(got == exp);
    Block back = CHBlockChunkCodecV1::decode(ctx, cb.cloneEmpty(), pk);
    EXPECT(back.getByName("d15").column->type == t15);
}

// DataTypeDecimal_test A (gtest_funtions_decimal_arith.cpp:47-77): Decimal(10,4) (+|-) Decimal(10,6)
// has scale max(4, 6) = 6 and Decimal(10,4) * Decimal(10,6) scale 4 + 6 = 10; precision per
// PlusDecimalInferer / MulDecimalInferer (Common/Decimal.h:109-163), values vs Int128 arithmetic.
TEST(DecimalArithInferers) {
    const size_t n = 1000;
    std::mt19937_64 rng(5);
    std::vector<int64_t> a(n), b(n);
    for (size_t i = 0; i < n; ++i) {
        a[i] = (int64_t)(rng() % 19999999999ull) - 9999999999ll; // |a| < 10^10: Decimal(10,4)
        b[i] = (int64_t)(rng() % 19999999999ull) - 9999999999ll;
    }
    DataType ta = DataType::decimal(10, 4), tb = DataType::decimal(10, 6);
    Block blk{{makeColumn(ctx, ta, a.data(), n), ta, "a"}, {makeColumn(ctx, tb, b.data(), n), tb, "b"}};
    auto e = std::make_shared<ExpressionActions>(ctx);
    e->arithmetic(TFG_PLUS, "a", "b", "p");
    e->arithmetic(TFG_MINUS, "a", "b", "m");
    e->arithmetic(TFG_MULTIPLY, "a", "b", "x");
    e->execute(blk);
    const IColumn &p = *blk.getByName("p").column, &m = *blk.getByName("m").column, &x = *blk.getByName("x").column;
    EXPECT(p.type.scale == 6 && m.type.scale == 6 && x.type.scale == 10);
    EXPECT(p.type.getName() == "Decimal(13,6)" && p.type.type == TFG_DECIMAL64);
    EXPECT(x.type.getName() == "Decimal(20,10)" && x.type.type == TFG_DECIMAL128);
    auto hp = toHost<int64_t>(ctx, p), hm = toHost<int64_t>(ctx, m);
    auto hx = toHost<__int128>(ctx, x);
    size_t bad = 0;
    for (size_t i = 0; i < n; ++i) {
        bad += hp[i] != a[i] * 100 + b[i];
        bad += hm[i] != a[i] * 100 - b[i];
        bad += hx[i] != (__int128)a[i] * b[i];
    }
    EXPECT(bad == 0);
}

// Past precision 38 the inferers give Decimal256 (createDecimal): Decimal(38,2) + Decimal(38,2) ->
// Decimal(39,2) and Decimal(20,16) * Decimal(20,16) -> Decimal(40,30), whose scale is capped at
// 30 (the product divided by 10^2, truncating); values vs __int128 arithmetic on small inputs.
TEST(DecimalArithDecimal256Results) {
    const size_t n = 777;
    std::mt19937_64 rng(9);
    std::vector<__int128> a(n), b(n);
    for (size_t i = 0; i < n; ++i) {
        a[i] = (__int128)((int64_t)(rng() >> 1) - (int64_t)(1ll << 61)) * 1000003;
        b[i] = (__int128)((int64_t)(rng() % 2000001) - 1000000);
    }
    DataType t38 = DataType::decimal(38, 2), t20 = DataType::decimal(20, 16);
    Block blk{{makeColumn(ctx, t38, a.data(), n), t38, "a"}, {makeColumn(ctx, t38, b.data(), n), t38, "b"},
              {makeColumn(ctx, t20, a.data(), n), t20, "c"}, {makeColumn(ctx, t20, b.data(), n), t20, "d"}};
    auto e = std::make_shared<ExpressionActions>(ctx);
    e->arithmetic(TFG_PLUS, "a", "b", "p");
    e->arithmetic(TFG_MULTIPLY, "c", "d", "x");
    e->execute(blk);
    const IColumn &p = *blk.getByName("p").column, &x = *blk.getByName("x").column;
    EXPECT(p.type.type == TFG_DECIMAL256 && p.type.getName() == "Decimal(39,2)");
    EXPECT(x.type.type == TFG_DECIMAL256 && x.type.getName() == "Decimal(40,30)");
    struct L4 {
        uint64_t w[4];
    };
    auto hp = toHost<L4>(ctx, p), hx = toHost<L4>(ctx, x);
    auto low128 = [](const L4 &v) { return (__int128)(((unsigned __int128)v.w[1] << 64) | v.w[0]); };
    auto ext_ok = [](const L4 &v) {
        const uint64_t s = (int64_t)v.w[1] < 0 ? ~0ull : 0ull;
        return v.w[2] == s && v.w[3] == s;
    };
    size_t bad = 0;
    for (size_t i = 0; i < n; ++i) {
        const __int128 prod = a[i] * b[i], q = prod / 100; // C++ division truncates toward zero
        bad += !ext_ok(hp[i]) || low128(hp[i]) != a[i] + b[i];
        bad += !ext_ok(hx[i]) || low128(hx[i]) != q;
    }
    EXPECT(bad == 0);
}

// ================================================================ pipeline engine (b)
// The reference's operator contract (Operators/Operator.h:32-173) driven the way its
// PipelineExec does (PipelineExec.cpp:120-180), two execs per pipeline, results vs the oracle.
static std::vector<Block> splitBlocks(Context &ctx, const Block &b, size_t parts) {
    std::vector<Block> out;
    const size_t n = b.rows();
    for (size_t i = 0; i < parts; ++i) {
        const size_t lo = n * i / parts, hi = n * (i + 1) / parts;
        out.push_back(sliceBlock(ctx, b, lo, hi - lo));
    }
    return out;
}

// filter -> aggregation: [BlocksSourceOp -> FilterTransformOp -> AggregateBuildSinkOp] x 2, then
// [AggregateConvergentSourceOp -> GetResultSinkOp] x 2; also the pushed-down (fused) filter form
TEST(PipelineFilterAggregate) {
    std::mt19937_64 rng(101);
    const size_t n = 200000;
    std::vector<int64_t> f(n), k(n);
    std::vector<double> d(n);
    for (size_t i = 0; i < n; ++i) {
        f[i] = rng() % 100;
        k[i] = (int64_t)(rng() % 30000);
        d[i] = (double)(rng() % (1 << 20)) / 256.0;
    }
    DataType i64, f64;
    f64.type = TFG_FLOAT64;
    Block b{{makeColumn(ctx, i64, f.data(), n), i64, "f"}, {makeColumn(ctx, i64, k.data(), n), i64, "k"},
            {makeColumn(ctx, f64, d.data(), n), f64, "d"}};
    std::vector<Block> blocks = splitBlocks(ctx, b, 6);
    Aggregator::Params p;
    p.src_header = b.cloneEmpty();
    p.keys = {"k"};
    p.aggregates = {{"sum", {"d"}, "sum_d"}, {"count", {}, "cnt"}};
    // oracle
    std::vector<uint8_t> mask(n);
    for (size_t i = 0; i < n; ++i) mask[i] = f[i] < 40;
    int kinds[2] = {TFG_AGG_SUM, TFG_AGG_COUNT_ALL};
    int types[2] = {TFG_FLOAT64, 0};
    orc_agg *o = orc_agg_create(TFG_INT64, 2, kinds, types);
    const void *args[2] = {d.data(), nullptr};
    const uint8_t *an[2] = {nullptr, nullptr};
    orc_agg_consume(o, k.data(), nullptr, args, an, mask.data(), n);
    const size_t g = orc_agg_size(o);
    std::vector<uint64_t> ok(g), oc(g);
    std::vector<double> od(g);
    std::vector<uint8_t> okn(g), on0(g), on1(g);
    void *outs[2] = {od.data(), oc.data()};
    uint8_t *outn[2] = {on0.data(), on1.data()};
    orc_agg_result(o, ok.data(), okn.data(), outs, outn);
    orc_agg_destroy(o);
    std::map<int64_t, std::pair<double, uint64_t>> want;
    for (size_t i = 0; i < g; ++i) want[(int64_t)ok[i]] = {od[i], oc[i]};
    for (int pushed = 0; pushed < 2; ++pushed) {
        g_current = pushed ? "pushed-down filter" : "FilterTransformOp";
        PipelineExecutorContext exec;
        auto agg_ctx = std::make_shared<AggregateContext>(ctx, p, 2);
        std::vector<PipelineExecPtr> build;
        for (size_t t = 0; t < 2; ++t) {
            std::vector<Block> mine;
            for (size_t i = t; i < blocks.size(); i += 2) mine.push_back(blocks[i]);
            TransformOps tr;
            auto sink = std::make_unique<AggregateBuildSinkOp>(exec, ctx, agg_ctx, t);
            if (pushed) {
                sink->setPushedDownFilter("f", TFG_LT, Field::Int64(40));
            } else {
                auto expr = std::make_shared<ExpressionActions>(ctx);
                expr->compare("f", TFG_LT, Field::Int64(40), "pred");
                Block h = b.cloneEmpty();
                tr.push_back(std::make_unique<FilterTransformOp>(exec, ctx, h, expr, "pred"));
            }
            build.push_back(std::make_unique<PipelineExec>(std::make_unique<BlocksSourceOp>(exec, ctx, b, mine),
                                                           std::move(tr), std::move(sink)));
        }
        runPipelineExecs(exec, build);
        EXPECT(agg_ctx->allBuildFinished());
        EXPECT(agg_ctx->getTotalBuildRows(0) + agg_ctx->getTotalBuildRows(1) == (pushed ? n : (size_t)std::count(mask.begin(), mask.end(), 1)));
        std::vector<Block> results;
        std::vector<PipelineExecPtr> conv;
        for (size_t t = 0; t < 2; ++t)
            conv.push_back(std::make_unique<PipelineExec>(
                std::make_unique<AggregateConvergentSourceOp>(exec, ctx, agg_ctx, t), TransformOps{},
                std::make_unique<GetResultSinkOp>(exec, ctx, [&](const Block &r) { results.push_back(r); })));
        runPipelineExecs(exec, conv);
        EXPECT(results.size() == 2); // one row range per convergent source
        std::map<int64_t, std::pair<double, uint64_t>> got;
        for (const Block &r : results) {
            auto rk = toHost<int64_t>(ctx, *r.getByName("k").column);
            auto rd = toHost<double>(ctx, *r.getByName("sum_d").column);
            auto rc = toHost<uint64_t>(ctx, *r.getByName("cnt").column);
            for (size_t i = 0; i < rk.size(); ++i) EXPECT(got.emplace(rk[i], std::make_pair(rd[i], rc[i])).second);
        }
        EXPECT(got == want);
        const auto &src = build[0]->source().getProfileInfo();
        EXPECT(src.blocks == 3 && src.rows == blocks[0].rows() + blocks[2].rows() + blocks[4].rows());
    }
}

// build -> probe: [BlocksSourceOp -> HashJoinBuildSink] x 2, then [BlocksSourceOp ->
// HashJoinProbeTransformOp (max_block_size 5000: output sliced through tryOutput) ->
// GetResultSinkOp] x 2, vs the oracle's pairs; also an empty build side
TEST(PipelineHashJoin) {
    std::mt19937_64 rng(102);
    const size_t nb = 40000, np = 120000;
    std::vector<int64_t> bk(nb), bp(nb), pk(np);
    for (size_t i = 0; i < nb; ++i) {
        bk[i] = rng() % 30000;
        bp[i] = (int64_t)i;
    }
    for (size_t i = 0; i < np; ++i) pk[i] = rng() % 50000;
    DataType i64;
    Block build{{makeColumn(ctx, i64, bk.data(), nb), i64, "bk"}, {makeColumn(ctx, i64, bp.data(), nb), i64, "bpay"}};
    Block probe{{makeColumn(ctx, i64, pk.data(), np), i64, "pk"}};
    orc_join *oj = orc_join_create(TFG_INT64);
    orc_join_build(oj, bk.data(), nullptr, nb);
    std::vector<uint32_t> op(np * 4), ob(np * 4);
    const size_t m = orc_join_probe(oj, TFG_JOIN_INNER, pk.data(), nullptr, np, op.data(), ob.data(), op.size());
    orc_join_destroy(oj);
    std::multiset<std::pair<int64_t, int64_t>> want;
    for (size_t i = 0; i < m; ++i) want.insert({pk[op[i]], bp[ob[i]]});
    for (int variant = 0; variant < 3; ++variant) {
        const int empty_build = variant == 1;
        g_current = variant == 0 ? "join" : variant == 1 ? "empty build" : "JoinV2 pointer table";
        PipelineExecutorContext exec;
        auto join = std::make_shared<Join>(ctx, JoinKind::Inner, "pk", "bk", (int64_t)nb);
        if (variant == 2) join->useJoinV2(true);
        auto jctx = std::make_shared<JoinBuildContext>(ctx, join, 2, build.cloneEmpty());
        std::vector<Block> bblocks = empty_build ? std::vector<Block>{} : splitBlocks(ctx, build, 4);
        std::vector<PipelineExecPtr> bpipe;
        for (size_t t = 0; t < 2; ++t) {
            std::vector<Block> mine;
            for (size_t i = t; i < bblocks.size(); i += 2) mine.push_back(bblocks[i]);
            bpipe.push_back(std::make_unique<PipelineExec>(std::make_unique<BlocksSourceOp>(exec, ctx, build, mine),
                                                           TransformOps{},
                                                           std::make_unique<HashJoinBuildSink>(exec, ctx, jctx, t)));
        }
        runPipelineExecs(exec, bpipe);
        EXPECT(jctx->isFinalized());
        std::vector<Block> pblocks = splitBlocks(ctx, probe, 3);
        std::vector<Block> out;
        std::vector<PipelineExecPtr> ppipe;
        for (size_t t = 0; t < 2; ++t) {
            std::vector<Block> mine;
            for (size_t i = t; i < pblocks.size(); i += 2) mine.push_back(pblocks[i]);
            TransformOps tr;
            auto probe_op = std::make_unique<HashJoinProbeTransformOp>(exec, ctx, jctx, t, 5000);
            Block h = probe.cloneEmpty();
            probe_op->transformHeader(h);
            tr.push_back(std::move(probe_op));
            ppipe.push_back(std::make_unique<PipelineExec>(std::make_unique<BlocksSourceOp>(exec, ctx, probe, mine),
                                                           std::move(tr),
                                                           std::make_unique<GetResultSinkOp>(exec, ctx, [&](const Block &r) {
                                                               out.push_back(r);
                                                           })));
        }
        runPipelineExecs(exec, ppipe);
        std::multiset<std::pair<int64_t, int64_t>> got;
        size_t max_rows = 0;
        for (const Block &r : out) {
            max_rows = std::max(max_rows, r.rows());
            auto gk = toHost<int64_t>(ctx, *r.getByName("pk").column);
            auto gb = toHost<int64_t>(ctx, *r.getByName("bpay").column);
            for (size_t i = 0; i < gk.size(); ++i) got.insert({gk[i], gb[i]});
        }
        if (empty_build) {
            EXPECT(got.empty());
        } else {
            EXPECT(got == want);
            EXPECT(max_rows <= 5000 && out.size() > 3); // sliced output
        }
    }
}

// exchange: [BlocksSourceOp -> ExchangeSenderSinkOp] x 2 into 4 partitions (partition 1 local,
// the others captured as remote tunnels), then [ExchangeReceiverSourceOp -> GetResultSinkOp];
// every partition's rows equal hashPartitionBlock's for the same input.  Then the one-rank MPP
// exchange (RCCL) path end to end.
TEST(PipelineExchange) {
    std::mt19937_64 rng(103);
    const size_t n = 50000;
    std::vector<int64_t> k(n), v(n);
    for (size_t i = 0; i < n; ++i) {
        k[i] = (int64_t)(rng() % 100000) - 50000;
        v[i] = (int64_t)i;
    }
    DataType i64;
    Block b{{makeColumn(ctx, i64, k.data(), n), i64, "k"}, {makeColumn(ctx, i64, v.data(), n), i64, "v"}};
    std::vector<Block> want = hashPartitionBlock(ctx, b, {0}, 4);
    std::vector<Block> blocks = splitBlocks(ctx, b, 5);
    PipelineExecutorContext exec;
    auto receiver = std::make_shared<ExchangeReceiver>();
    std::vector<std::multiset<std::vector<std::string>>> remote(4);
    auto tunnels = std::make_shared<MPPTunnelSet>(ctx, 4, 2, receiver, nullptr, 1, [&](uint32_t part, Block &&blk, uint32_t) {
        for (const auto &row : rowSet(ctx, blk)) remote[part].insert(row);
    });
    std::vector<PipelineExecPtr> send;
    for (size_t t = 0; t < 2; ++t) {
        std::vector<Block> mine;
        for (size_t i = t; i < blocks.size(); i += 2) mine.push_back(blocks[i]);
        send.push_back(std::make_unique<PipelineExec>(std::make_unique<BlocksSourceOp>(exec, ctx, b, mine), TransformOps{},
                                                      std::make_unique<ExchangeSenderSinkOp>(exec, ctx, tunnels,
                                                                                             std::vector<size_t>{0})));
    }
    runPipelineExecs(exec, send);
    EXPECT(receiver->finished());
    std::multiset<std::vector<std::string>> local;
    std::vector<PipelineExecPtr> recv;
    recv.push_back(std::make_unique<PipelineExec>(
        std::make_unique<ExchangeReceiverSourceOp>(exec, ctx, receiver, b), TransformOps{},
        std::make_unique<GetResultSinkOp>(exec, ctx, [&](const Block &r) {
            for (const auto &row : rowSet(ctx, r)) local.insert(row);
        })));
    runPipelineExecs(exec, recv);
    EXPECT(local == rowSet(ctx, want[1]));
    for (uint32_t p : {0u, 2u, 3u}) EXPECT(remote[p] == rowSet(ctx, want[p]));
    // one-rank MPP exchange: everything comes back
    uint8_t id[128];
    check(tfg_comm_unique_id(id, sizeof(id)), "tfg_comm_unique_id");
    MPPExchange mpp(ctx, 1, 0, id, sizeof(id));
    auto recv1 = std::make_shared<ExchangeReceiver>();
    auto t1 = std::make_shared<MPPTunnelSet>(ctx, 1, 1, recv1, &mpp);
    std::vector<PipelineExecPtr> s1;
    s1.push_back(std::make_unique<PipelineExec>(std::make_unique<BlocksSourceOp>(exec, ctx, b, blocks), TransformOps{},
                                                std::make_unique<ExchangeSenderSinkOp>(exec, ctx, t1, std::vector<size_t>{0})));
    runPipelineExecs(exec, s1);
    Block all;
    EXPECT(recv1->tryPop(all) && rowSet(ctx, all) == rowSet(ctx, b));
}

// PipelineExec's contract: a cancelled context stops execute() with CANCELLED (the reference's
// SimpleOperatorTestRunner.cancel); an operator returning a status outside its contract throws;
// a filter that empties a block asks for more input (NEED_INPUT) instead of passing it on.
TEST(PipelineExecContract) {
    DataType i64;
    std::vector<int64_t> x = {1, 2, 3};
    Block b{{makeColumn(ctx, i64, x.data(), 3), i64, "x"}};
    {
        PipelineExecutorContext exec;
        PipelineExec pe(std::make_unique<BlocksSourceOp>(exec, ctx, b, std::vector<Block>{b}), TransformOps{},
                        std::make_unique<GetResultSinkOp>(exec, ctx, [](const Block &) {}));
        exec.cancel();
        EXPECT(pe.execute() == OperatorStatus::CANCELLED);
    }
    {
        PipelineExecutorContext exec;
        auto expr = std::make_shared<ExpressionActions>(ctx);
        expr->compare("x", TFG_GT, Field::Int64(10), "pred"); // filters every row
        TransformOps tr;
        tr.push_back(std::make_unique<FilterTransformOp>(exec, ctx, b.cloneEmpty(), expr, "pred"));
        size_t seen = 0;
        PipelineExec pe(std::make_unique<BlocksSourceOp>(exec, ctx, b, std::vector<Block>{b, b}), std::move(tr),
                        std::make_unique<GetResultSinkOp>(exec, ctx, [&](const Block &) { ++seen; }));
        EXPECT(pe.execute() == OperatorStatus::NEED_INPUT);
        EXPECT(pe.execute() == OperatorStatus::NEED_INPUT);
        EXPECT(pe.execute() == OperatorStatus::FINISHED); // the end-of-input block reaches the sink
        EXPECT(seen == 0);
    }
    {
        struct BadSource : SourceOp {
            using SourceOp::SourceOp;
            std::string getName() const override { return "BadSource"; }
            OperatorStatus readImpl(Block &) override { return OperatorStatus::NEED_INPUT; }
        };
        PipelineExecutorContext exec;
        PipelineExec pe(std::make_unique<BadSource>(exec, ctx), TransformOps{},
                        std::make_unique<GetResultSinkOp>(exec, ctx, [](const Block &) {}));
        bool threw = false;
        try {
            pe.execute();
        } catch (const Exception &) {
            threw = true;
        }
        EXPECT(threw);
    }
    { // a selective block into an operator that cannot take one
        PipelineExecutorContext exec;
        Block sb = b;
        sb.info.selective = makeSelective(ctx, {0, 2});
        PipelineExec pe(std::make_unique<BlocksSourceOp>(exec, ctx, b, std::vector<Block>{sb}), TransformOps{},
                        std::make_unique<GetResultSinkOp>(exec, ctx, [](const Block &) {}));
        bool threw = false;
        try {
            pe.execute();
        } catch (const Exception &) {
            threw = true;
        }
        EXPECT(threw);
    }
}

// BlockInfo::selective through the exchange (gtest_mpp_exchange_writer.cpp:1147-1230): the
// partitions of a selective block hold exactly the selected rows, each where a full-block
// partition puts it (selective hash = full hash at the same rows), String and Nullable columns
// included, through hashPartitionBlock and HashPartitionWriter
TEST(SelectiveBlockPartition) {
    std::mt19937_64 rng(104);
    const size_t n = 4096, ns = 1024;
    std::vector<int64_t> k(n), v(n);
    std::vector<uint8_t> kn(n);
    std::vector<std::string> s(n);
    for (size_t i = 0; i < n; ++i) {
        k[i] = (int64_t)(rng() % 3000);
        v[i] = (int64_t)i;
        kn[i] = rng() % 13 == 0;
        s[i] = "s" + std::to_string(rng() % 500) + std::string(rng() % 20, 'x');
    }
    std::vector<uint64_t> sel;
    for (size_t i = 0; i < n && sel.size() < ns; ++i)
        if (rng() % 4 == 0 || n - i <= ns - sel.size()) sel.push_back(i);
    DataType i64, i64n, str{DataType::TYPE_STRING};
    i64n.nullable = true;
    for (int with_string = 0; with_string < 2; ++with_string) {
        g_current = with_string ? "string key" : "int key";
        Block b{{makeColumn(ctx, i64n, k.data(), n, kn.data()), i64n, "k"}, {makeColumn(ctx, i64, v.data(), n), i64, "v"}};
        if (with_string) b.insert({makeStringColumn(ctx, s), str, "s"});
        const std::vector<size_t> keys = with_string ? std::vector<size_t>{2, 0} : std::vector<size_t>{0};
        std::vector<Block> full = hashPartitionBlock(ctx, b, keys, 4);
        Block sb = b;
        sb.info.selective = makeSelective(ctx, sel);
        std::vector<Block> part = hashPartitionBlock(ctx, sb, keys, 4);
        std::set<int64_t> chosen(sel.begin(), sel.end());
        size_t total = 0;
        for (uint32_t p = 0; p < 4; ++p) {
            auto fv = toHost<int64_t>(ctx, *full[p].getByName("v").column);
            std::vector<int64_t> expect_v;
            for (int64_t x : fv)
                if (chosen.count(x)) expect_v.push_back(x); // same partition, same (stable) order
            auto pv = toHost<int64_t>(ctx, *part[p].getByName("v").column);
            EXPECT(pv == expect_v);
            total += pv.size();
            if (with_string) EXPECT(part[p].getByName("s").column->rows == pv.size());
        }
        EXPECT(total == ns);
        // HashPartitionWriter: only the listed rows are sent
        std::vector<std::vector<int64_t>> sent(4);
        HashPartitionWriter w(ctx, keys, 4, [&](uint32_t p, Block &&blk) {
            auto pv = toHost<int64_t>(ctx, *blk.getByName("v").column);
            sent[p].insert(sent[p].end(), pv.begin(), pv.end());
        });
        w.write(sb);
        w.flush();
        for (uint32_t p = 0; p < 4; ++p) EXPECT(sent[p] == toHost<int64_t>(ctx, *part[p].getByName("v").column));
    }
}

// ---------------------------------------------------------------- executor descriptors (row b2)
// PhysicalPlan::build (Flash/Planner/PhysicalPlan.cpp:95-231) from tipb-shaped descriptors: the
// operators are instantiated by the planner, not by hand, and the results equal the oracle's.
static std::map<int64_t, std::pair<double, uint64_t>> planAggRows(Context &ctx, const std::vector<Block> &res) {
    std::map<int64_t, std::pair<double, uint64_t>> got;
    for (const Block &r : res) { // schema: sum, count, key
        auto rs = toHost<double>(ctx, *r.safeGetByPosition(0).column);
        auto rc = toHost<uint64_t>(ctx, *r.safeGetByPosition(1).column);
        auto rk = toHost<int64_t>(ctx, *r.safeGetByPosition(2).column);
        for (size_t i = 0; i < rk.size(); ++i) EXPECT(got.emplace(rk[i], std::make_pair(rs[i], rc[i])).second);
    }
    return got;
}

// Aggregation(Selection(TableScan)): filter -> GROUP BY from a descriptor, both with the pushed-down
// (fused) filter and with FilterTransformOp, through the pipeline engine and the stream engine;
// then computed arguments: sum(d * 2.0) and sum(100 - f) (a constant-left MinusInt)
TEST(PlanFilterAggregate) {
    using namespace dag;
    std::mt19937_64 rng(201);
    const size_t n = 150000;
    std::vector<int64_t> f(n), k(n);
    std::vector<double> d(n);
    for (size_t i = 0; i < n; ++i) {
        f[i] = rng() % 100;
        k[i] = (int64_t)(rng() % 20000) - 5000;
        d[i] = (double)(rng() % (1 << 20)) / 256.0;
    }
    DataType i64, f64;
    f64.type = TFG_FLOAT64;
    Block b{{makeColumn(ctx, i64, f.data(), n), i64, "f"}, {makeColumn(ctx, i64, k.data(), n), i64, "k"},
            {makeColumn(ctx, f64, d.data(), n), f64, "d"}};
    std::map<int64_t, std::pair<double, uint64_t>> want;
    std::map<int64_t, int64_t> want_minus;
    for (size_t i = 0; i < n; ++i)
        if (f[i] < 40) {
            auto &w = want[k[i]];
            w.first += d[i];
            w.second += 1;
            want_minus[k[i]] += 100 - f[i];
        }
    // oracle check of the host map (dyadic values: exact in any order)
    {
        std::vector<uint8_t> mask(n);
        for (size_t i = 0; i < n; ++i) mask[i] = f[i] < 40;
        int kinds[2] = {TFG_AGG_SUM, TFG_AGG_COUNT_ALL};
        int types[2] = {TFG_FLOAT64, 0};
        orc_agg *o = orc_agg_create(TFG_INT64, 2, kinds, types);
        const void *args[2] = {d.data(), nullptr};
        const uint8_t *an[2] = {nullptr, nullptr};
        orc_agg_consume(o, k.data(), nullptr, args, an, mask.data(), n);
        EXPECT(orc_agg_size(o) == want.size());
        orc_agg_destroy(o);
    }
    PlanContext env;
    env.tables["lineitem"] = {b.cloneEmpty(), splitBlocks(ctx, b, 5)};
    const Executor root = Executor::aggregation(
        "agg_1", {Expr::col(1)}, {Expr::sum(Expr::col(2)), Expr::count()},
        Executor::selection("sel_0", {Expr::func(ScalarFuncSig::LTInt, {Expr::col(0), Expr::i64(40)})},
                            Executor::tableScan("ts_0", "lineitem")));
    for (int fuse = 0; fuse < 2; ++fuse) {
        g_current = fuse ? "PlanFilterAggregate fused" : "PlanFilterAggregate FilterTransformOp";
        std::vector<Block> res;
        env.result = [&](const Block &r) { res.push_back(r); };
        env.fuse_filter_into_aggregation = fuse;
        PipelineExecutorContext exec;
        PhysicalPlan plan(ctx, exec, env);
        plan.build(root);
        const std::string shape = plan.toString();
        EXPECT(plan.pipelines().size() == 2);
        EXPECT((shape.find("FilterTransformOp") != std::string::npos) == !fuse);
        EXPECT(shape.find("AggregateBuildSinkOp x2") != std::string::npos);
        EXPECT(shape.find("AggregateConvergentSourceOp") != std::string::npos);
        EXPECT(plan.outputHeader().columns() == 3);
        plan.execute();
        EXPECT(planAggRows(ctx, res) == want);
    }
    { // the stream engine's chain of the same descriptor
        g_current = "PlanFilterAggregate streams";
        BlockInputStreamPtr s = buildBlockInputStream(ctx, env, root);
        std::vector<Block> res;
        for (Block r = s->read(); r; r = s->read()) res.push_back(r);
        EXPECT(planAggRows(ctx, res) == want);
    }
    { // computed arguments: sum(d * 2.0), sum(100 - f), count(*)
        g_current = "PlanFilterAggregate computed args";
        const Executor r2 = Executor::aggregation(
            "agg_2", {Expr::col(1)},
            {Expr::sum(Expr::func(ScalarFuncSig::MultiplyReal, {Expr::col(2), Expr::f64(2.0)})),
             Expr::count(), Expr::sum(Expr::func(ScalarFuncSig::MinusInt, {Expr::i64(100), Expr::col(0)}))},
            Executor::selection("sel_0", {Expr::func(ScalarFuncSig::GTInt, {Expr::i64(40), Expr::col(0)})},
                                Executor::tableScan("ts_0", "lineitem")));
        std::vector<Block> res;
        env.result = [&](const Block &r) { res.push_back(r); };
        env.fuse_filter_into_aggregation = true;
        PipelineExecutorContext exec;
        PhysicalPlan plan(ctx, exec, env);
        plan.build(r2);
        EXPECT(plan.toString().find("ExpressionTransformOp") != std::string::npos);
        plan.execute();
        std::map<int64_t, std::pair<double, uint64_t>> got;
        std::map<int64_t, int64_t> got_minus;
        for (const Block &r : res) { // schema: sum(d*2), count, sum(100-f), key
            auto rs = toHost<double>(ctx, *r.safeGetByPosition(0).column);
            auto rc = toHost<uint64_t>(ctx, *r.safeGetByPosition(1).column);
            auto rm = toHost<int64_t>(ctx, *r.safeGetByPosition(2).column);
            auto rk = toHost<int64_t>(ctx, *r.safeGetByPosition(3).column);
            for (size_t i = 0; i < rk.size(); ++i) {
                got[rk[i]] = {rs[i] / 2.0, rc[i]};
                got_minus[rk[i]] = rm[i];
            }
        }
        EXPECT(got == want);
        EXPECT(got_minus == want_minus);
        if (got != want || got_minus != want_minus) { // bisect: the same aggregation without the planner
            auto ea = std::make_shared<ExpressionActions>(ctx);
            ea->arithmeticConst(TFG_MULTIPLY, "d", Field::Float64(2.0), "x2");
            ea->arithmeticConstLeft(TFG_MINUS, Field::Int64(100), "f", "m");
            Block bx = b;
            ea->execute(bx);
            Aggregator::Params p2;
            p2.src_header = bx.cloneEmpty();
            p2.keys = {"k"};
            p2.aggregates = {{"sum", {"x2"}, "s"}, {"count", {}, "c"}, {"sum", {"m"}, "sm"}};
            Aggregator direct(ctx, p2);
            direct.executeOnBlockFiltered(bx, "f", TFG_LT, Field::Int64(40));
            Block r = direct.convertToBlock();
            auto rk = toHost<int64_t>(ctx, *r.getByName("k").column);
            auto rs = toHost<double>(ctx, *r.getByName("s").column);
            auto rc = toHost<uint64_t>(ctx, *r.getByName("c").column);
            std::map<int64_t, std::pair<double, uint64_t>> g2;
            for (size_t i = 0; i < rk.size(); ++i) g2[rk[i]] = {rs[i] / 2.0, rc[i]};
            fprintf(stderr, "  direct Aggregator (no planner): %s, groups %zu; block rows %zu, cols %zu\n",
                    g2 == want ? "matches" : "differs", g2.size(), bx.rows(), bx.columns());
        }
        if (got != want || got_minus != want_minus) { // diagnostics: the first differing groups
            fprintf(stderr, "  groups got %zu want %zu\n", got.size(), want.size());
            int shown = 0;
            for (const auto &kv : want) {
                auto it = got.find(kv.first);
                auto im = got_minus.find(kv.first);
                const bool bad = it == got.end() || it->second != kv.second || im == got_minus.end() ||
                                 im->second != want_minus[kv.first];
                if (bad && shown++ < 5)
                    fprintf(stderr, "  key %lld: want (%.6f, %llu, %lld) got (%.6f, %llu, %lld)\n", (long long)kv.first,
                            kv.second.first, (unsigned long long)kv.second.second, (long long)want_minus[kv.first],
                            it == got.end() ? -1.0 : it->second.first,
                            it == got.end() ? 0ull : (unsigned long long)it->second.second,
                            im == got_minus.end() ? -1ll : (long long)im->second);
            }
        }
    }
}

// min / max / first_row through the planner (tipb Min / Max / First) and through a two-phase
// Aggregator: min(Nullable Int32), max(Float64), first_row of a column that depends on the key,
// first_row of the key itself (agg_func_ref_key: the key column, Nullable), count(*); checked
// against host maps built with the reference's semantics (AggregateFunctionMinMaxAny.h).
TEST(PlanAggregateMinMaxFirstRow) {
    using namespace dag;
    std::mt19937_64 rng(77);
    const size_t n = 120000;
    std::vector<int64_t> k(n);
    std::vector<int32_t> v(n);
    std::vector<uint8_t> vn(n);
    std::vector<double> x(n);
    std::vector<int16_t> y(n);
    for (size_t i = 0; i < n; ++i) {
        k[i] = (int64_t)(rng() % 3000) - 1000;
        v[i] = (int32_t)(rng() % 2000001) - 1000000;
        vn[i] = (k[i] % 7 == 0) || (rng() % 4 == 0); // every row NULL for keys divisible by 7
        x[i] = (double)((int64_t)(rng() % (1 << 24)) - (1 << 23)) / 64.0;
        y[i] = (int16_t)(k[i] % 1000);
    }
    DataType i64, i32n, f64, i16;
    i32n.type = TFG_INT32;
    i32n.nullable = true;
    f64.type = TFG_FLOAT64;
    i16.type = TFG_INT16;
    Block b{{makeColumn(ctx, i64, k.data(), n), i64, "k"}, {makeColumn(ctx, i32n, v.data(), n, vn.data()), i32n, "v"},
            {makeColumn(ctx, f64, x.data(), n), f64, "x"}, {makeColumn(ctx, i16, y.data(), n), i16, "y"}};
    struct W {
        bool has_v = false;
        int32_t mn = 0;
        double mx = 0;
        uint64_t cnt = 0;
    };
    std::map<int64_t, W> want;
    for (size_t i = 0; i < n; ++i) {
        W &w = want[k[i]];
        if (!vn[i] && (!w.has_v || v[i] < w.mn)) w.mn = v[i], w.has_v = true; // changeIfLess
        if (w.cnt == 0 || x[i] > w.mx) w.mx = x[i];                              // changeIfGreater
        ++w.cnt;
    }
    // one output row -> its cells as strings (min v, max x, first_row y, first_row k, count, key)
    auto rows = [&](const std::vector<Block> &res, int ci_min, int ci_max, int ci_fy, int ci_fk, int ci_cnt, int ci_key) {
        std::map<int64_t, std::vector<std::string>> got;
        for (const Block &r : res) {
            auto mn = cellStrings(ctx, *materialize(ctx, r.safeGetByPosition(ci_min).column));
            auto mx = toHost<double>(ctx, *r.safeGetByPosition(ci_max).column);
            auto fy = cellStrings(ctx, *materialize(ctx, r.safeGetByPosition(ci_fy).column));
            auto fk = cellStrings(ctx, *materialize(ctx, r.safeGetByPosition(ci_fk).column));
            auto cn = toHost<uint64_t>(ctx, *r.safeGetByPosition(ci_cnt).column);
            auto kk = toHost<int64_t>(ctx, *r.safeGetByPosition(ci_key).column);
            EXPECT(r.safeGetByPosition(ci_min).type.nullable && r.safeGetByPosition(ci_fk).type.nullable);
            EXPECT(!r.safeGetByPosition(ci_max).type.nullable && r.safeGetByPosition(ci_fy).type.type == TFG_INT16);
            for (size_t i = 0; i < kk.size(); ++i)
                got[kk[i]] = {mn[i], std::to_string(mx[i]), fy[i], fk[i], std::to_string(cn[i])};
        }
        return got;
    };
    std::map<int64_t, std::vector<std::string>> expect;
    for (const auto &kv : want)
        expect[kv.first] = {kv.second.has_v ? std::to_string(kv.second.mn) : "N", std::to_string(kv.second.mx),
                            std::to_string(kv.first % 1000), std::to_string(kv.first), std::to_string(kv.second.cnt)};
    { // the planner: Aggregation(group by k: min(v), max(x), first_row(y), first_row(k), count(*))
        g_current = "PlanAggregateMinMaxFirstRow plan";
        PlanContext env;
        env.tables["t"] = {b.cloneEmpty(), splitBlocks(ctx, b, 4)};
        const Executor root = Executor::aggregation(
            "agg_1", {Expr::col(0)},
            {Expr::min(Expr::col(1)), Expr::max(Expr::col(2)), Expr::firstRow(Expr::col(3)), Expr::firstRow(Expr::col(0)),
             Expr::count()},
            Executor::tableScan("ts_0", "t"));
        std::vector<Block> res;
        env.result = [&](const Block &r) { res.push_back(r); };
        PipelineExecutorContext exec;
        PhysicalPlan plan(ctx, exec, env);
        plan.build(root);
        EXPECT(plan.outputHeader().columns() == 6);
        plan.execute();
        EXPECT(rows(res, 0, 1, 2, 3, 4, 5) == expect);
    }
    { // two phases: partial blocks of two halves merged by a final aggregator (mergeOnBlock)
        g_current = "PlanAggregateMinMaxFirstRow two-phase";
        Aggregator::Params p;
        p.src_header = b.cloneEmpty();
        p.keys = {"k"};
        p.aggregates = {{"min", {"v"}, "mn"}, {"max", {"x"}, "mx"}, {"first_row", {"y"}, "fy"},
                        {"first_row", {"k"}, "fk"}, {"count", {}, "c"}};
        std::vector<Block> halves = splitBlocks(ctx, b, 2);
        Aggregator fin(ctx, p);
        for (const Block &h : halves) {
            Aggregator part(ctx, p);
            part.executeOnBlock(h);
            Block pb = part.convertToBlock(false);
            fin.mergeOnBlock(pb);
        }
        Block r = fin.convertToBlock();
        auto got = rows({r}, 1, 2, 3, 4, 5, 0);
        // the merged count is a sum of partial counts
        EXPECT(got == expect);
        if (got != expect) { // the first difference, for the log
            size_t shown = 0;
            for (const auto &kv : expect) {
                auto it = got.find(kv.first);
                if (it != got.end() && it->second == kv.second) continue;
                std::string g = it == got.end() ? "(missing)" : "", e;
                if (it != got.end())
                    for (auto &x : it->second) g += x + " ";
                for (auto &x : kv.second) e += x + " ";
                fprintf(stderr, "    key %lld: got %s want %s\n", (long long)kv.first, g.c_str(), e.c_str());
                if (++shown == 5) break;
            }
            fprintf(stderr, "    groups got %zu want %zu\n", got.size(), expect.size());
        }
    }
    { // only key references: a hidden count keeps the device aggregator
        g_current = "PlanAggregateMinMaxFirstRow key references only";
        Aggregator::Params p;
        p.src_header = b.cloneEmpty();
        p.keys = {"k"};
        p.aggregates = {{"first_row", {"k"}, "fk"}};
        Aggregator agg(ctx, p);
        agg.executeOnBlock(b);
        Block r = agg.convertToBlock();
        EXPECT(r.columns() == 2);
        auto kk = toHost<int64_t>(ctx, *r.getByName("k").column);
        auto fk = cellStrings(ctx, *materialize(ctx, r.getByName("fk").column));
        EXPECT(kk.size() == want.size());
        bool same = kk.size() == fk.size();
        for (size_t i = 0; same && i < kk.size(); ++i) same = fk[i] == std::to_string(kk[i]);
        EXPECT(same);
    }
}

static std::multiset<std::vector<std::string>> byteRowSet(Context &ctx, const Block &b);

// min / max / first_row over String (under general_ci and binary) and Decimal128 through the planner
// (one PipelineExec: blocks in order, so first_row is the first row) and the Aggregator's two
// phases, against a host restatement: SingleValueDataString / SingleValueDataFixed strict
// changeIfLess / changeIfGreater / changeFirstTime, the collator's compare over the row with its
// '\0' (orc_min_max_str_compare), a NULL first row NULL (AggregateFunctionMinMaxAny.cpp:46,85,98,155)
TEST(PlanAggregateWideMinMaxFirstRow) {
    using namespace dag;
    std::mt19937_64 rng(91);
    const size_t n = 60000;
    const char *alpha[] = {"a", "A", "b", "B", " ", "\xc3\xa9", "\xc3\x89", "ss", "\xc3\x9f", "z"};
    std::vector<int64_t> k(n);
    std::vector<std::string> s(n);
    std::vector<uint8_t> sn(n);
    std::vector<__int128> d(n);
    for (size_t i = 0; i < n; ++i) {
        k[i] = (int64_t)(rng() % 2000);
        for (size_t j = 0, len = rng() % 4; j < len; ++j) s[i] += alpha[rng() % 10];
        sn[i] = rng() % 5 == 0;
        d[i] = ((__int128)((int64_t)(rng() % 200) - 100) << 70) + (__int128)(rng() % 3);
    }
    DataType i64, str_n, dec = DataType::decimal(38, 2);
    str_n.type = DataType::TYPE_STRING;
    str_n.nullable = true;
    Block b{{makeColumn(ctx, i64, k.data(), n), i64, "k"}, {makeStringColumn(ctx, s, sn.data()), str_n, "s"},
            {makeColumn(ctx, dec, d.data(), n), dec, "d"}};
    auto hex = [](const __int128 &v) {
        static const char hx[] = "0123456789abcdef";
        std::string o;
        const uint8_t *p = (const uint8_t *)&v;
        for (int q = 0; q < 16; ++q) o.push_back(hx[p[q] >> 4]), o.push_back(hx[p[q] & 15]);
        return o;
    };
    auto cmp = [](int coll, const std::string &a, const std::string &b) {
        return orc_min_max_str_compare(coll, (const uint8_t *)a.c_str(), a.size() + 1, (const uint8_t *)b.c_str(), b.size() + 1);
    };
    struct W {
        bool mn_has = false, mx_has = false, first = false, first_null = false;
        std::string mn, mx, fs;
        __int128 fd = 0;
    };
    std::map<int64_t, W> want;
    for (size_t i = 0; i < n; ++i) {
        W &w = want[k[i]];
        if (!w.first) w.first = true, w.first_null = sn[i], w.fs = s[i], w.fd = d[i];
        if (!sn[i] && (!w.mn_has || cmp(TFG_COLLATOR_GENERAL_CI, s[i], w.mn) < 0)) w.mn = s[i], w.mn_has = true;
        if (!sn[i] && (!w.mx_has || cmp(TFG_COLLATOR_NONE, s[i], w.mx) > 0)) w.mx = s[i], w.mx_has = true;
    }
    // max(d) per key: a separate pass (strict: the first maximum)
    std::map<int64_t, __int128> dmx;
    for (size_t i = 0; i < n; ++i) {
        auto it = dmx.find(k[i]);
        if (it == dmx.end() || d[i] > it->second) dmx[k[i]] = d[i];
    }
    std::multiset<std::vector<std::string>> expect, expect2;
    for (const auto &kv : want) {
        const W &w = kv.second;
        int64_t key = kv.first;
        std::string khex;
        static const char hx[] = "0123456789abcdef";
        for (int q = 0; q < 8; ++q) {
            const uint8_t byte = (uint8_t)((uint64_t)key >> (8 * q));
            khex.push_back(hx[byte >> 4]), khex.push_back(hx[byte & 15]);
        }
        expect.insert({w.mn_has ? w.mn : "N", w.mx_has ? w.mx : "N", w.first_null ? "N" : w.fs, hex(dmx[key]), khex});
        expect2.insert({hex(w.fd), w.first_null ? "N" : w.fs, khex});
    }
    { // Aggregation(group by k: min(s) general_ci, max(s), first_row(s), max(d), first_row(d))
        g_current = "PlanAggregateWideMinMaxFirstRow plan";
        PlanContext env;
        env.concurrency = 1;
        env.tables["t"] = {b.cloneEmpty(), splitBlocks(ctx, b, 3)};
        const Executor root = Executor::aggregation(
            "agg_1", {Expr::col(0)},
            {Expr::min(Expr::col(1), TFG_COLLATOR_GENERAL_CI), Expr::max(Expr::col(1)), Expr::firstRow(Expr::col(1)),
             Expr::max(Expr::col(2))},
            Executor::tableScan("ts_0", "t"));
        std::vector<Block> res;
        env.result = [&](const Block &r) { res.push_back(r); };
        PipelineExecutorContext exec;
        PhysicalPlan plan(ctx, exec, env);
        plan.build(root);
        plan.execute();
        std::multiset<std::vector<std::string>> got;
        for (const Block &r : res) {
            EXPECT(r.safeGetByPosition(0).type.isString() && r.safeGetByPosition(0).type.nullable);
            EXPECT(r.safeGetByPosition(2).type.nullable && r.safeGetByPosition(3).type.type == TFG_DECIMAL128);
            for (const auto &row : byteRowSet(ctx, r)) got.insert(row);
        }
        EXPECT(got == expect);
    }
    { // two phases: partial blocks of three slices merged in order by a final aggregator
        g_current = "PlanAggregateWideMinMaxFirstRow two-phase";
        Aggregator::Params p;
        p.src_header = b.cloneEmpty();
        p.keys = {"k"};
        AggregateDescription mn{"min", {"s"}, "mn"};
        mn.collator = TFG_COLLATOR_GENERAL_CI;
        p.aggregates = {mn, {"max", {"s"}, "mx"}, {"first_row", {"s"}, "fs"}, {"max", {"d"}, "md"}};
        Aggregator::Params p2 = p;
        p2.aggregates = {{"first_row", {"d"}, "fd"}, {"first_row", {"s"}, "fs"}};
        for (int which = 0; which < 2; ++which) {
            Aggregator fin(ctx, which ? p2 : p);
            for (const Block &h : splitBlocks(ctx, b, 3)) {
                Aggregator part(ctx, which ? p2 : p);
                part.executeOnBlock(h);
                fin.mergeOnBlock(part.convertToBlock(false));
            }
            Block r = fin.convertToBlock();
            // byteRowSet orders the columns as the block does: key first here
            std::multiset<std::vector<std::string>> got;
            for (auto row : byteRowSet(ctx, r)) {
                std::rotate(row.begin(), row.begin() + 1, row.end());
                got.insert(row);
            }
            EXPECT(got == (which ? expect2 : expect));
        }
    }
}

// Join(TableScan probe, TableScan build) from descriptors: inner (pairs vs the oracle, schema =
// left then right columns), a GROUP BY over the join (count per key), left outer (unmatched
// probe rows carry NULL build columns), semi, and the stream engine's inner join
TEST(PlanHashJoin) {
    using namespace dag;
    std::mt19937_64 rng(202);
    const size_t nb = 30000, np = 90000;
    std::vector<int64_t> bk(nb), bp(nb), pk(np), pp(np);
    for (size_t i = 0; i < nb; ++i) {
        bk[i] = rng() % 25000;
        bp[i] = (int64_t)i * 7;
    }
    for (size_t i = 0; i < np; ++i) {
        pk[i] = rng() % 40000;
        pp[i] = (int64_t)i;
    }
    DataType i64;
    Block build{{makeColumn(ctx, i64, bk.data(), nb), i64, "o_key"}, {makeColumn(ctx, i64, bp.data(), nb), i64, "o_pay"}};
    Block probe{{makeColumn(ctx, i64, pk.data(), np), i64, "l_key"}, {makeColumn(ctx, i64, pp.data(), np), i64, "l_pay"}};
    orc_join *oj = orc_join_create(TFG_INT64);
    orc_join_build(oj, bk.data(), nullptr, nb);
    std::vector<uint32_t> op(np * 4), ob(np * 4);
    const size_t m = orc_join_probe(oj, TFG_JOIN_INNER, pk.data(), nullptr, np, op.data(), ob.data(), op.size());
    orc_join_destroy(oj);
    std::multiset<std::vector<int64_t>> want;
    std::map<int64_t, uint64_t> want_cnt;
    std::vector<uint8_t> matched(np, 0);
    for (size_t i = 0; i < m; ++i) {
        want.insert({pk[op[i]], pp[op[i]], bk[ob[i]], bp[ob[i]]});
        ++want_cnt[pk[op[i]]];
        matched[op[i]] = 1;
    }
    const size_t unmatched = (size_t)std::count(matched.begin(), matched.end(), 0);
    PlanContext env;
    env.tables["lineitem"] = {probe.cloneEmpty(), splitBlocks(ctx, probe, 4)};
    env.tables["orders"] = {build.cloneEmpty(), splitBlocks(ctx, build, 3)};
    env.max_block_size = 20000;
    auto joinOf = [&](JoinType t) {
        return Executor::join("join_2", t, {Expr::col(0)}, {Expr::col(0)}, Executor::tableScan("ts_0", "lineitem"),
                              Executor::tableScan("ts_1", "orders"), 1);
    };
    auto rows4 = [&](const std::vector<Block> &res) {
        std::multiset<std::vector<int64_t>> got;
        for (const Block &r : res) {
            std::vector<std::vector<int64_t>> c;
            for (size_t j = 0; j < 4; ++j) c.push_back(toHost<int64_t>(ctx, *r.safeGetByPosition(j).column));
            for (size_t i = 0; i < c[0].size(); ++i) got.insert({c[0][i], c[1][i], c[2][i], c[3][i]});
        }
        return got;
    };
    { // inner
        g_current = "PlanHashJoin inner";
        std::vector<Block> res;
        env.result = [&](const Block &r) { res.push_back(r); };
        PipelineExecutorContext exec;
        PhysicalPlan plan(ctx, exec, env);
        plan.build(joinOf(JoinType::TypeInnerJoin));
        EXPECT(plan.pipelines().size() == 2);
        EXPECT(plan.toString().find("HashJoinBuildSink x2") != std::string::npos);
        EXPECT(plan.toString().find("HashJoinProbeTransformOp") != std::string::npos);
        EXPECT(plan.outputHeader().columns() == 4 && plan.outputHeader().safeGetByPosition(0).name == "join_2_l_l_key" &&
               plan.outputHeader().safeGetByPosition(2).name == "join_2_r_o_key");
        plan.execute();
        EXPECT(rows4(res) == want);
        size_t max_rows = 0;
        for (const Block &r : res) max_rows = std::max(max_rows, r.rows());
        EXPECT(max_rows <= 20000);
    }
    { // GROUP BY the joined key: count(*) per l_key
        g_current = "PlanHashJoin aggregation over the join";
        std::vector<Block> res;
        env.result = [&](const Block &r) { res.push_back(r); };
        PipelineExecutorContext exec;
        PhysicalPlan plan(ctx, exec, env);
        plan.build(Executor::aggregation("agg_3", {Expr::col(0)}, {Expr::count()}, joinOf(JoinType::TypeInnerJoin)));
        EXPECT(plan.pipelines().size() == 3); // join build, probe -> agg build, convergent
        plan.execute();
        std::map<int64_t, uint64_t> got;
        for (const Block &r : res) {
            auto rc = toHost<uint64_t>(ctx, *r.safeGetByPosition(0).column);
            auto rk = toHost<int64_t>(ctx, *r.safeGetByPosition(1).column);
            for (size_t i = 0; i < rk.size(); ++i) got[rk[i]] = rc[i];
        }
        EXPECT(got == want_cnt);
    }
    { // left outer: every probe row, unmatched ones with NULL build columns
        g_current = "PlanHashJoin left outer";
        std::vector<Block> res;
        env.result = [&](const Block &r) { res.push_back(r); };
        PipelineExecutorContext exec;
        PhysicalPlan plan(ctx, exec, env);
        plan.build(joinOf(JoinType::TypeLeftOuterJoin));
        EXPECT(plan.outputHeader().safeGetByPosition(3).type.nullable);
        plan.execute();
        size_t rows = 0, nulls = 0;
        for (const Block &r : res) {
            rows += r.rows();
            auto nm = toHostNullMap(ctx, *r.safeGetByPosition(3).column);
            nulls += (size_t)std::count(nm.begin(), nm.end(), 1);
        }
        EXPECT(rows == m + unmatched && nulls == unmatched);
    }
    { // semi: the probe rows with a match (left columns only)
        g_current = "PlanHashJoin semi";
        std::vector<Block> res;
        env.result = [&](const Block &r) { res.push_back(r); };
        PipelineExecutorContext exec;
        PhysicalPlan plan(ctx, exec, env);
        plan.build(joinOf(JoinType::TypeSemiJoin));
        EXPECT(plan.outputHeader().columns() == 2);
        plan.execute();
        std::multiset<int64_t> got, exp;
        for (const Block &r : res)
            for (int64_t v : toHost<int64_t>(ctx, *r.safeGetByPosition(1).column)) got.insert(v);
        for (size_t i = 0; i < np; ++i)
            if (matched[i]) exp.insert(pp[i]);
        EXPECT(got == exp);
    }
    { // the stream engine
        g_current = "PlanHashJoin streams";
        BlockInputStreamPtr s = buildBlockInputStream(ctx, env, joinOf(JoinType::TypeInnerJoin));
        std::vector<Block> res;
        for (Block r = s->read(); r; r = s->read()) res.push_back(r);
        EXPECT(rows4(res) == want);
    }
}

// ExchangeSender(Hash) -> tunnels (partition 1 local, the others captured), vs hashPartitionBlock;
// then ExchangeReceiver -> Aggregation on the local partition; PassThrough and Broadcast senders
TEST(PlanExchange) {
    using namespace dag;
    std::mt19937_64 rng(203);
    const size_t n = 40000;
    std::vector<int64_t> k(n), v(n);
    for (size_t i = 0; i < n; ++i) {
        k[i] = (int64_t)(rng() % 5000) - 2500;
        v[i] = (int64_t)(rng() % 1000);
    }
    DataType i64;
    Block b{{makeColumn(ctx, i64, k.data(), n), i64, "k"}, {makeColumn(ctx, i64, v.data(), n), i64, "v"}};
    std::vector<Block> want = hashPartitionBlock(ctx, b, {0}, 4);
    PlanContext env;
    env.tables["t"] = {b.cloneEmpty(), splitBlocks(ctx, b, 5)};
    auto receiver = std::make_shared<ExchangeReceiver>();
    std::vector<std::multiset<std::vector<std::string>>> remote(4);
    env.tunnels = std::make_shared<MPPTunnelSet>(ctx, 4, 2, receiver, nullptr, 1, [&](uint32_t part, Block &&blk, uint32_t) {
        for (const auto &row : rowSet(ctx, blk)) remote[part].insert(row);
    });
    {
        PipelineExecutorContext exec;
        PhysicalPlan plan(ctx, exec, env);
        plan.build(Executor::exchangeSender("exchange_sender_1", ExchangeType::Hash, {Expr::col(0)},
                                            Executor::tableScan("ts_0", "t")));
        EXPECT(plan.toString().find("ExchangeSenderSinkOp x2") != std::string::npos);
        plan.execute();
    }
    EXPECT(receiver->finished());
    for (uint32_t p : {0u, 2u, 3u}) EXPECT(remote[p] == rowSet(ctx, want[p]));
    // the receiving task: GROUP BY k over the local partition
    std::map<int64_t, std::pair<int64_t, uint64_t>> exp;
    {
        auto wk = toHost<int64_t>(ctx, *want[1].safeGetByPosition(0).column);
        auto wv = toHost<int64_t>(ctx, *want[1].safeGetByPosition(1).column);
        for (size_t i = 0; i < wk.size(); ++i) {
            exp[wk[i]].first += wv[i];
            exp[wk[i]].second += 1;
        }
    }
    PlanContext env2;
    env2.receivers["exchange_receiver_0"] = {b.cloneEmpty(), receiver};
    std::vector<Block> res;
    env2.result = [&](const Block &r) { res.push_back(r); };
    {
        PipelineExecutorContext exec;
        PhysicalPlan plan(ctx, exec, env2);
        plan.build(Executor::aggregation("agg_1", {Expr::col(0)}, {Expr::sum(Expr::col(1)), Expr::count()},
                                         Executor::exchangeReceiver("exchange_receiver_0", "exchange_receiver_0")));
        EXPECT(plan.toString().find("ExchangeReceiverSourceOp") != std::string::npos);
        plan.execute();
    }
    std::map<int64_t, std::pair<int64_t, uint64_t>> got;
    for (const Block &r : res) {
        auto rs = toHost<int64_t>(ctx, *r.safeGetByPosition(0).column);
        auto rc = toHost<uint64_t>(ctx, *r.safeGetByPosition(1).column);
        auto rk = toHost<int64_t>(ctx, *r.safeGetByPosition(2).column);
        for (size_t i = 0; i < rk.size(); ++i) got[rk[i]] = {rs[i], rc[i]};
    }
    EXPECT(got == exp);
    // PassThrough: every row to tunnel 0; Broadcast: every row to every tunnel
    for (int bc = 0; bc < 2; ++bc) {
        g_current = bc ? "PlanExchange broadcast" : "PlanExchange pass-through";
        std::vector<size_t> rows(3, 0);
        auto recv = std::make_shared<ExchangeReceiver>();
        PlanContext e3;
        e3.tables["t"] = env.tables["t"];
        e3.tunnels = std::make_shared<MPPTunnelSet>(ctx, 3, 2, recv, nullptr, 0,
                                                    [&](uint32_t part, Block &&blk, uint32_t) { rows[part] += blk.rows(); });
        PipelineExecutorContext exec;
        PhysicalPlan plan(ctx, exec, e3);
        plan.build(Executor::exchangeSender("exchange_sender_2", bc ? ExchangeType::Broadcast : ExchangeType::PassThrough,
                                            {}, Executor::tableScan("ts_0", "t")));
        plan.execute();
        size_t local = 0;
        for (Block blk; recv->tryPop(blk);) local += blk ? blk.rows() : 0;
        EXPECT(local == n);
        EXPECT(bc ? (rows[1] == n && rows[2] == n) : (rows[1] == 0 && rows[2] == 0));
    }
}

// ExchangeSender with fine_grained_shuffle_stream_count = 4 from a descriptor: the sink op runs a
// FineGrainedShuffleWriter; the local partition's blocks reach the receiver tagged with their
// streams (every row of stream s has weak hash % 4 == s and partition 0), the remote partition's
// rows are the partition's rows, and a fine-grained receiver plan (concurrency 4, one stream per
// source) aggregates the local partition exactly.
TEST(PlanExchangeFineGrained) {
    using namespace dag;
    std::mt19937_64 rng(204);
    const size_t n = 30000;
    const uint32_t P = 2, S = 4;
    std::vector<int64_t> k(n), v(n);
    for (size_t i = 0; i < n; ++i) {
        k[i] = (int64_t)(rng() % 4000) - 2000;
        v[i] = (int64_t)(rng() % 1000);
    }
    DataType i64;
    Block b{{makeColumn(ctx, i64, k.data(), n), i64, "k"}, {makeColumn(ctx, i64, v.data(), n), i64, "v"}};
    auto part_of = [&](int64_t x, uint32_t &stream) {
        const uint32_t h = orc_crc32c_u64(0xFFFFFFFFu, (uint64_t)x);
        stream = h % S;
        return (uint32_t)(((uint64_t)h * P) >> 32);
    };
    std::map<int64_t, std::pair<int64_t, uint64_t>> exp_local;
    size_t remote_want = 0;
    for (size_t i = 0; i < n; ++i) {
        uint32_t s;
        if (part_of(k[i], s) == 0) {
            exp_local[k[i]].first += v[i];
            exp_local[k[i]].second += 1;
        } else {
            ++remote_want;
        }
    }
    std::set<uint32_t> remote_streams;
    auto run_sender = [&](std::shared_ptr<ExchangeReceiver> receiver, size_t &remote_rows) {
        PlanContext env;
        env.tables["t"] = {b.cloneEmpty(), splitBlocks(ctx, b, 6)};
        env.tunnels = std::make_shared<MPPTunnelSet>(
            ctx, P, 2, receiver, nullptr, 0, [&](uint32_t part, Block &&blk, uint32_t stream) {
                EXPECT(part == 1);
                remote_rows += blk.rows();
                // the remote partition's blocks keep their streams: every row of the block has
                // weak hash % S == stream (fillSelectorForFineGrainedShuffle)
                bool ok = stream < S;
                for (int64_t x : toHost<int64_t>(ctx, *blk.getByName("k").column)) {
                    uint32_t s2;
                    ok = ok && part_of(x, s2) == 1 && s2 == stream;
                }
                EXPECT(ok);
                remote_streams.insert(stream);
            });
        Executor root = Executor::exchangeSender("exchange_sender_1", ExchangeType::Hash, {Expr::col(0)},
                                                 Executor::tableScan("ts_0", "t"));
        root.fine_grained_shuffle_stream_count = S;
        root.fine_grained_shuffle_batch_size = 1000;
        PipelineExecutorContext exec;
        PhysicalPlan plan(ctx, exec, env);
        plan.build(root);
        plan.execute();
        EXPECT(receiver->finished());
    };
    { // the streams as the receiver holds them
        g_current = "PlanExchangeFineGrained streams";
        auto receiver = std::make_shared<ExchangeReceiver>();
        size_t remote_rows = 0;
        run_sender(receiver, remote_rows);
        EXPECT(remote_rows == remote_want);
        EXPECT(remote_streams.size() == S); // every stream reached the remote partition
        size_t local_rows = 0;
        for (uint32_t s = 0; s < S; ++s)
            for (Block blk; receiver->tryPop(blk, S, s);) {
                std::vector<int64_t> kk = toHost<int64_t>(ctx, *blk.getByName("k").column);
                for (int64_t x : kk) {
                    uint32_t st;
                    EXPECT(part_of(x, st) == 0 && st == s);
                }
                local_rows += kk.size();
            }
        EXPECT(local_rows == n - remote_want);
    }
    { // a fine-grained receiver plan: GROUP BY k over the local partition, one stream per source
        g_current = "PlanExchangeFineGrained receiver plan";
        auto receiver = std::make_shared<ExchangeReceiver>();
        size_t remote_rows = 0;
        run_sender(receiver, remote_rows);
        PlanContext env2;
        env2.concurrency = S;
        env2.receivers["exchange_receiver_0"] = {b.cloneEmpty(), receiver};
        std::vector<Block> res;
        env2.result = [&](const Block &r) { res.push_back(r); };
        Executor recv = Executor::exchangeReceiver("exchange_receiver_0", "exchange_receiver_0");
        recv.fine_grained_shuffle_stream_count = S;
        PipelineExecutorContext exec;
        PhysicalPlan plan(ctx, exec, env2);
        plan.build(Executor::aggregation("agg_1", {Expr::col(0)}, {Expr::sum(Expr::col(1)), Expr::count()}, recv));
        plan.execute();
        std::map<int64_t, std::pair<int64_t, uint64_t>> got;
        for (const Block &r : res) {
            auto rs = toHost<int64_t>(ctx, *r.safeGetByPosition(0).column);
            auto rc = toHost<uint64_t>(ctx, *r.safeGetByPosition(1).column);
            auto rk = toHost<int64_t>(ctx, *r.safeGetByPosition(2).column);
            for (size_t i = 0; i < rk.size(); ++i) got[rk[i]] = {rs[i], rc[i]};
        }
        EXPECT(got == exp_local);
    }
}

// ================================================================ two ranks over TCP
// The MPPExchange transport seam: a host-staged TCP transport between two test processes
// (test infrastructure; the product's transport is RcclTransport).  Rank 0 listens on
// 127.0.0.1:port, rank 1 connects.  Counts and bytes cross as host buffers; a rank's own slice is a
// device copy.  Rank 0 writes before it reads, rank 1 reads before it writes (no write/write stall).
class TcpTransport : public ExchangeTransport {
public:
    TcpTransport(Context &ctx, int rank, int port) : ctx_(ctx), rank_(rank) {
        if (rank == 0) {
            const int ls = ::socket(AF_INET, SOCK_STREAM, 0);
            int one = 1;
            ::setsockopt(ls, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
            sockaddr_in a{};
            a.sin_family = AF_INET;
            a.sin_port = htons((uint16_t)port);
            a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
            if (::bind(ls, (sockaddr *)&a, sizeof a) || ::listen(ls, 1)) throw std::runtime_error("bind/listen");
            fd_ = ::accept(ls, nullptr, nullptr);
            ::close(ls);
        } else {
            for (int attempt = 0; attempt < 600 && fd_ < 0; ++attempt) {
                const int c = ::socket(AF_INET, SOCK_STREAM, 0);
                sockaddr_in a{};
                a.sin_family = AF_INET;
                a.sin_port = htons((uint16_t)port);
                a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
                if (::connect(c, (sockaddr *)&a, sizeof a) == 0) fd_ = c;
                else {
                    ::close(c);
                    usleep(100000);
                }
            }
        }
        if (fd_ < 0) throw std::runtime_error("tcp transport: no peer");
    }
    ~TcpTransport() override {
        if (fd_ >= 0) ::close(fd_);
    }
    int nranks() const override { return 2; }
    int rank() const override { return rank_; }
    void alltoallCountsN(int k, const uint64_t *send, uint64_t *recv) override {
        std::vector<uint64_t> peer(2 * (size_t)k);
        swap(send, sizeof(uint64_t) * 2 * k, peer.data(), peer.size() * sizeof(uint64_t));
        for (int i = 0; i < k; ++i) {
            recv[(size_t)rank_ * k + i] = send[(size_t)rank_ * k + i];
            recv[(size_t)(1 - rank_) * k + i] = peer[(size_t)rank_ * k + i];
        }
    }
    // the peer's slices in order through one host buffer each way; this rank's own by device copies
    void exchangeSlices(const std::vector<tfg_slice> &send, const std::vector<tfg_slice> &recv) override {
        const int q = 1 - rank_;
        std::vector<uint8_t> out, in;
        for (const tfg_slice &sl : send)
            if (sl.peer == q && sl.bytes) {
                const size_t o = out.size();
                out.resize(o + sl.bytes);
                check(tfg_download(ctx_.raw(), out.data() + o, sl.ptr, sl.bytes), "tfg_download");
            }
        size_t in_bytes = 0;
        for (const tfg_slice &sl : recv)
            if (sl.peer == q) in_bytes += sl.bytes;
        in.resize(in_bytes);
        swap(out.data(), out.size(), in.data(), in.size());
        size_t o = 0;
        for (const tfg_slice &sl : recv)
            if (sl.peer == q && sl.bytes) {
                check(tfg_upload(ctx_.raw(), sl.ptr, in.data() + o, sl.bytes), "tfg_upload");
                o += sl.bytes;
            }
        std::vector<const tfg_slice *> mine_s, mine_r; // own slices: k-th send -> k-th receive
        for (const tfg_slice &sl : send)
            if (sl.peer == rank_ && sl.bytes) mine_s.push_back(&sl);
        for (const tfg_slice &sl : recv)
            if (sl.peer == rank_ && sl.bytes) mine_r.push_back(&sl);
        if (mine_s.size() != mine_r.size()) throw std::runtime_error("own slices do not match");
        for (size_t i = 0; i < mine_s.size(); ++i) {
            if (mine_s[i]->bytes != mine_r[i]->bytes) throw std::runtime_error("own slice sizes differ");
            check(tfg_copy(ctx_.raw(), mine_r[i]->ptr, mine_s[i]->ptr, mine_s[i]->bytes), "tfg_copy");
        }
    }

private:
    Context &ctx_;
    int rank_, fd_ = -1;
    void put(const void *p, size_t n) {
        for (size_t d = 0; d < n;) {
            const ssize_t w = ::write(fd_, (const char *)p + d, n - d);
            if (w <= 0) throw std::runtime_error("tcp write");
            d += (size_t)w;
        }
    }
    void get(void *p, size_t n) {
        for (size_t d = 0; d < n;) {
            const ssize_t r = ::read(fd_, (char *)p + d, n - d);
            if (r <= 0) throw std::runtime_error("tcp read");
            d += (size_t)r;
        }
    }
    void swap(const void *out, size_t n_out, void *in, size_t n_in) {
        if (rank_ == 0) {
            put(out, n_out);
            get(in, n_in);
        } else {
            get(in, n_in);
            put(out, n_out);
        }
    }
};

// Rank r's input of case c (deterministic, so each rank can rebuild its peer's rows): c = 0 fixed
// columns (Int64 key, Nullable Int32 with and without a null map, Decimal(30,2) as 16-byte values,
// Float64), c = 1 String key + Int64, c = 2 fixed columns with rank 1 sending no rows at all.
static Block exchangeInput(Context &ctx, int c, int r) {
    std::mt19937_64 rng(1000 * c + r + 1);
    const size_t n = (c == 2 && r == 1) ? 0 : 20000 + 3000 * r;
    std::vector<int64_t> k(std::max<size_t>(n, 1)), f(std::max<size_t>(n, 1));
    std::vector<int32_t> v(std::max<size_t>(n, 1));
    std::vector<uint8_t> vn(std::max<size_t>(n, 1));
    std::vector<int64_t> dec(2 * std::max<size_t>(n, 1));
    std::vector<double> x(std::max<size_t>(n, 1));
    std::vector<std::string> strs;
    for (size_t i = 0; i < n; ++i) {
        k[i] = (int64_t)(rng() % 7000) - 3000;
        v[i] = (int32_t)(rng() % 100000);
        vn[i] = rng() % 5 == 0;
        dec[2 * i] = (int64_t)(rng() >> 2);
        dec[2 * i + 1] = (int64_t)(rng() % 3) - 1;
        x[i] = (double)(rng() % (1 << 20)) / 8.0;
        f[i] = (int64_t)i;
        strs.push_back("s" + std::to_string(rng() % 5000) + (rng() % 2 ? "_tail_beyond_16_bytes" : ""));
    }
    DataType i64, i32n, d30, f64, str;
    i32n.type = TFG_INT32;
    i32n.nullable = true;
    d30 = DataType::decimal(30, 2);
    f64.type = TFG_FLOAT64;
    str.type = DataType::TYPE_STRING;
    if (c == 1) {
        return Block{{makeStringColumn(ctx, strs), str, "s"},
                     {makeColumn(ctx, i64, f.data(), n), i64, "f"}};
    }
    DataType i32n_nomap = i32n; // a Nullable column that carries no null map on this rank
    return Block{{makeColumn(ctx, i64, k.data(), n), i64, "k"},
                 {makeColumn(ctx, i32n, v.data(), n, vn.data()), i32n, "v"},
                 {r == 0 ? makeColumn(ctx, i32n_nomap, v.data(), n) : makeColumn(ctx, i32n, v.data(), n, vn.data()),
                  i32n, "w"},
                 {makeColumn(ctx, d30, dec.data(), n), d30, "d"},
                 {makeColumn(ctx, f64, x.data(), n), f64, "x"}};
}

// rows as tuples of cell bytes (hex), any width, Strings as their text, NULL as "N"
static std::multiset<std::vector<std::string>> byteRowSet(Context &ctx, const Block &b) {
    std::vector<std::vector<std::string>> cols;
    for (const auto &cw : b.getColumnsWithTypeAndName()) {
        ColumnPtr c = materialize(ctx, cw.column);
        std::vector<std::string> out(c->rows);
        const std::vector<uint8_t> nm = toHostNullMap(ctx, *c);
        if (c->type.isString()) {
            out = toHostStrings(ctx, *c);
        } else {
            const std::vector<uint8_t> v = toHostBytes(ctx, *c);
            const size_t w = c->type.width();
            static const char hx[] = "0123456789abcdef";
            for (size_t i = 0; i < c->rows; ++i)
                for (size_t k = 0; k < w; ++k) {
                    out[i].push_back(hx[v[i * w + k] >> 4]);
                    out[i].push_back(hx[v[i * w + k] & 15]);
                }
        }
        for (size_t i = 0; i < c->rows; ++i)
            if (!nm.empty() && nm[i]) out[i] = "N";
        cols.push_back(std::move(out));
    }
    std::multiset<std::vector<std::string>> rows;
    for (size_t r = 0; r < b.rows(); ++r) {
        std::vector<std::string> t;
        for (auto &c : cols) t.push_back(c[r]);
        rows.insert(t);
    }
    return rows;
}

// rank: exchange each case's partition-major blocks with the peer; what arrives must be, as a row
// multiset, partition `rank` of both ranks' inputs (the oracle's routing: weak hash of column 0)
static int runExchangeRank(Context &ctx, int rank, int port) {
    auto t = std::make_shared<TcpTransport>(ctx, rank, port);
    MPPExchange ex(ctx, t);
    int bad = 0;
    for (int c = 0; c < 3; ++c) {
        g_current = "exchange case " + std::to_string(c) + " rank " + std::to_string(rank);
        std::vector<Block> parts = hashPartitionBlock(ctx, exchangeInput(ctx, c, rank), {0}, 2);
        Block got = ex.exchange(parts);
        std::multiset<std::vector<std::string>> want;
        for (int r = 0; r < 2; ++r) {
            Block in = exchangeInput(ctx, c, r);
            if (!in.rows()) continue;
            for (const auto &row : byteRowSet(ctx, hashPartitionBlock(ctx, in, {0}, 2)[rank])) want.insert(row);
        }
        const auto have = byteRowSet(ctx, got);
        const int before = g_failures;
        EXPECT(got.columns() == parts[0].columns());
        EXPECT(have == want);
        printf("[%s] exchange case %d rank %d: %zu rows\n", g_failures == before ? "  OK  " : " FAIL ", c, rank,
               (size_t)got.rows());
        bad += g_failures != before;
    }
    return bad ? 1 : 0;
}

// a crash names its test and where it happened (stdout into a pipe is lost with the process)
static void onFatalSignal(int sig) {
    const char *head = "  FATAL signal in ";
    (void)!write(2, head, strlen(head));
    (void)!write(2, g_current.data(), g_current.size());
    (void)!write(2, "\n", 1);
    void *frames[64];
    backtrace_symbols_fd(frames, backtrace(frames, 64), 2);
    signal(sig, SIG_DFL);
    raise(sig);
}

int main(int argc, char **argv) {
    setvbuf(stdout, nullptr, _IOLBF, 0);
    signal(SIGSEGV, onFatalSignal);
    signal(SIGABRT, onFatalSignal);
    signal(SIGBUS, onFatalSignal);
    g_root = argc > 1 ? argv[1] : ".";
    const char *filter = argc > 2 ? argv[2] : nullptr;
    std::unique_ptr<Context> owned;
    try {
        owned = std::make_unique<Context>(0);
    } catch (const Exception &e) {
        fprintf(stderr, "no device: %s\n", e.what());
        return 2;
    }
    Context &ctx = *owned;
    if (filter && !strcmp(filter, "--exchange-rank")) { // test_host <root> --exchange-rank <rank> <port>
        if (argc < 5) return 2;
        try {
            return runExchangeRank(ctx, atoi(argv[3]), atoi(argv[4]));
        } catch (const std::exception &e) {
            fprintf(stderr, "  EXCEPTION in exchange rank: %s\n", e.what());
            return 1;
        }
    }
    int failed_tests = 0, ran = 0;
    for (const auto &t : registry()) {
        if (filter && !strstr(t.name, filter)) continue;
        const int before = g_failures;
        g_current = t.name;
        try {
            t.fn(ctx);
        } catch (const std::exception &e) {
            ++g_failures;
            fprintf(stderr, "  EXCEPTION in %s [%s]: %s\n", t.name, g_current.c_str(), e.what());
        }
        ++ran;
        const bool ok = g_failures == before;
        failed_tests += !ok;
        printf("[%s] %s\n", ok ? "  OK  " : " FAIL ", t.name);
    }
    printf("%d tests, %d failed\n", ran, failed_tests);
    return failed_tests ? 1 : 0;
}
