// History ingest (include/jh_io.h): history.edn / test.fressian -> the
// columnar layout of jh.h, on the host, in native code.
//
// Reference: jepsen/src/jepsen/store.clj:346-357 (write-history!, one
// prn-printed op map per line via util.clj:191-213 pwrite-history!) and
// :359-366 / :177-183 (test.fressian, written and read with the handlers of
// store.clj:28-123 on top of clojure.data.fressian's). The encoding rules are
// jepsen_amd/history.py `encode` (tests/test_ingest.py holds this file to it).
//
// EDN: the bytes are split into one chunk per thread at line starts; every
// chunk is parsed speculatively (a chunk boundary is a form boundary when the
// previous chunk's last form ends exactly there, which is checked; a chunk
// that started inside a form is re-parsed sequentially). Each chunk interns
// processes, :f names, keys (and values, when some value is not an integer)
// in a local table; the tables are merged in chunk order, which is history
// order, so every id is the first-appearance id a sequential pass gives.
// fressian: one sequential pass (its priority and struct caches are state
// carried through the stream); the :history vector is streamed op by op.
#include "../../include/jh_io.h"

#include <algorithm>
#include <chrono>
#include <cerrno>
#include <numeric>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fcntl.h>
#include <string>
#include <string_view>
#include <sys/mman.h>
#include <sys/stat.h>
#include <thread>
#include <unistd.h>
#include <unordered_map>
#include <vector>

namespace {

// ---------------------------------------------------------------------------
// parsed values (both formats build these; one arena per thread, reset per op)
enum : uint8_t { V_NIL, V_TRUE, V_FALSE, V_INT, V_FLOAT, V_STR, V_KW, V_SYM, V_VEC, V_SET, V_MAP, V_TAG, V_RATIO, V_OPAQUE };

struct Val {
    uint8_t k;
    uint8_t src;            // text lives in the input bytes at (const char *)i
    uint32_t a, n;          // text: offset/len in txt; collection: offset/count in kids
    int64_t i;
    double d;
};

struct Arena {
    std::vector<Val> v;
    std::vector<uint32_t> kids, stk;
    std::string txt;
    void reset() { v.clear(); kids.clear(); txt.clear(); stk.clear(); }
    uint32_t leaf(uint8_t k, int64_t i = 0, double d = 0) {
        v.push_back(Val{k, 0, 0, 0, i, d});
        return (uint32_t)v.size() - 1;
    }
    uint32_t text(uint8_t k, const char *s, size_t n) {
        uint32_t off = (uint32_t)txt.size();
        txt.append(s, n);
        v.push_back(Val{k, 0, off, (uint32_t)n, 0, 0});
        return (uint32_t)v.size() - 1;
    }
    // text referenced in place (the EDN input outlives the parse)
    uint32_t srctext(uint8_t k, const char *s, size_t n) {
        v.push_back(Val{k, 1, 0, (uint32_t)n, (int64_t)(intptr_t)s, 0});
        return (uint32_t)v.size() - 1;
    }
    // children pushed on stk since `base` become the collection's kids
    uint32_t coll(uint8_t k, size_t base, uint32_t textoff = 0, uint32_t textlen = 0) {
        uint32_t off = (uint32_t)kids.size();
        uint32_t n = (uint32_t)(stk.size() - base);
        kids.insert(kids.end(), stk.begin() + base, stk.end());
        stk.resize(base);
        v.push_back(Val{k, 0, off, n, (int64_t)textoff, (double)textlen});
        return (uint32_t)v.size() - 1;
    }
    std::string_view sv(uint32_t x) const {
        return v[x].src ? std::string_view((const char *)(intptr_t)v[x].i, v[x].n)
                        : std::string_view(txt.data() + v[x].a, v[x].n);
    }
    uint32_t kid(uint32_t x, uint32_t j) const { return kids[v[x].a + j]; }
    // V_TAG keeps its tag text in (i, d) = (offset, length)
    std::string_view tag(uint32_t x) const { return std::string_view(txt.data() + v[x].i, (size_t)v[x].d); }
};

// deep copy between arenas (fressian cache entries outlive the per-op arena)
uint32_t copy_tree(const Arena &s, uint32_t x, Arena &d) {
    const Val &e = s.v[x];
    switch (e.k) {
    case V_STR: case V_KW: case V_SYM: case V_RATIO: case V_OPAQUE: {
        std::string_view t = s.sv(x);
        return d.text(e.k, t.data(), t.size());
    }
    case V_VEC: case V_SET: case V_MAP: case V_TAG: {
        uint32_t toff = 0, tlen = 0;
        if (e.k == V_TAG) { toff = (uint32_t)d.txt.size(); tlen = (uint32_t)e.d; d.txt.append(s.tag(x)); }
        std::vector<uint32_t> ch(e.n);
        for (uint32_t j = 0; j < e.n; j++) ch[j] = copy_tree(s, s.kids[e.a + j], d);
        size_t base = d.stk.size();
        d.stk.insert(d.stk.end(), ch.begin(), ch.end());
        return d.coll(e.k, base, toff, tlen);
    }
    default: return d.leaf(e.k, e.i, e.d);
    }
}

// ---------------------------------------------------------------------------
// canonical EDN text: the identity of a value for interning (with a class
// prefix mirroring Python's (type name, value) keys in history.encode) and
// the text handed back through jh_ingest_table_entry (edn.read_all reads it
// back into the object history.encode would have kept).
void put_str(std::string &o, std::string_view s) {
    o.push_back('"');
    for (unsigned char c : s) {
        switch (c) {
        case '"': o += "\\\""; break;
        case '\\': o += "\\\\"; break;
        case '\n': o += "\\n"; break;
        case '\t': o += "\\t"; break;
        case '\r': o += "\\r"; break;
        default:
            if (c < 0x20) { char b[8]; snprintf(b, sizeof b, "\\u%04x", c); o += b; }
            else o.push_back((char)c);
        }
    }
    o.push_back('"');
}

void put_float(std::string &o, double d) {
    char b[40];
    snprintf(b, sizeof b, "%.17g", d);
    o += b;
    if (!strpbrk(b, ".eEni")) o += ".0";
}

void canon(const Arena &A, uint32_t x, std::string &o, bool map_key = false) {
    const Val &e = A.v[x];
    switch (e.k) {
    case V_NIL: o += "nil"; break;
    case V_TRUE: o += "true"; break;
    case V_FALSE: o += "false"; break;
    case V_INT: o += std::to_string(e.i); break;
    case V_FLOAT: put_float(o, e.d); break;
    case V_STR: put_str(o, A.sv(x)); break;
    case V_KW:
        if (map_key) put_str(o, A.sv(x));      // edn.py: keyword map keys become str
        else { o.push_back(':'); o += A.sv(x); }
        break;
    case V_SYM: case V_RATIO: case V_OPAQUE: o += A.sv(x); break;
    case V_VEC:
        o.push_back('[');
        for (uint32_t j = 0; j < e.n; j++) { if (j) o.push_back(' '); canon(A, A.kid(x, j), o); }
        o.push_back(']');
        break;
    case V_SET: {
        std::vector<std::string> el(e.n);
        for (uint32_t j = 0; j < e.n; j++) canon(A, A.kid(x, j), el[j]);
        std::sort(el.begin(), el.end());
        o += "#{";
        for (uint32_t j = 0; j < e.n; j++) { if (j) o.push_back(' '); o += el[j]; }
        o.push_back('}');
        break;
    }
    case V_MAP:
        o.push_back('{');
        for (uint32_t j = 0; j + 1 < e.n + 1 && j < e.n; j += 2) {
            if (j) o += ", ";
            canon(A, A.kid(x, j), o, true);
            o.push_back(' ');
            if (j + 1 < e.n) canon(A, A.kid(x, j + 1), o);
        }
        o.push_back('}');
        break;
    case V_TAG:
        o.push_back('#');
        o += A.tag(x);
        o.push_back(' ');
        if (e.n == 1) canon(A, A.kid(x, 0), o);
        else {
            o.push_back('[');
            for (uint32_t j = 0; j < e.n; j++) { if (j) o.push_back(' '); canon(A, A.kid(x, j), o); }
            o.push_back(']');
        }
        break;
    }
}

char vclass(uint8_t k) {
    switch (k) {
    case V_INT: return 'i';
    case V_FLOAT: return 'f';
    case V_STR: return 's';
    case V_KW: return 'k';
    case V_SYM: return 'y';
    case V_VEC: return 'l';
    case V_SET: return 'z';
    case V_MAP: return 'd';
    case V_TAG: return 't';
    case V_RATIO: return 'r';
    case V_TRUE: case V_FALSE: return 'b';
    case V_NIL: return 'n';
    default: return 'o';
    }
}

// value identity (history.encode's `scalar`: (type name, value))
std::string value_ident(const Arena &A, uint32_t x) {
    std::string s(1, vclass(A.v[x].k));
    canon(A, x, s);
    return s;
}

// dict-key identity (process / :f / key): edn.py hands keywords over as str,
// and a Keyword equals the str of its name in Python, so both share class 's'
std::string name_ident(const Arena &A, uint32_t x) {
    const Val &e = A.v[x];
    if (e.k == V_KW || e.k == V_STR) { std::string s = "s"; s += A.sv(x); return s; }
    return value_ident(A, x);
}

// the text a table entry is handed back as (process / :f names are str)
std::string name_text(const Arena &A, uint32_t x) {
    std::string o;
    if (A.v[x].k == V_KW) put_str(o, A.sv(x));
    else canon(A, x, o);
    return o;
}

struct LocalTable {
    std::unordered_map<std::string, uint32_t> ids;
    std::unordered_map<int64_t, uint32_t> int_ids;   // integer entries (the common key / value)
    std::vector<std::string> ident, text;
    uint32_t get_int(int64_t v) {
        auto it = int_ids.find(v);
        if (it != int_ids.end()) return it->second;
        std::string t = std::to_string(v);
        uint32_t id = get("i" + t, t);
        int_ids.emplace(v, id);
        return id;
    }
    uint32_t get(std::string &&id, const std::string &txt) {
        auto it = ids.find(id);
        if (it != ids.end()) return it->second;
        uint32_t n = (uint32_t)ident.size();
        ids.emplace(id, n);
        ident.push_back(std::move(id));
        text.push_back(txt);
        return n;
    }
};

struct IoErr {
    int code = JH_OK;
    std::string msg;
    size_t at = 0;          // byte offset
};

// ---------------------------------------------------------------------------
// EDN reader: the subset prn emits (maps, vectors, lists, sets, keywords,
// symbols, strings, chars, integers, ratios, floats, nil/true/false, #tag
// literals, #_ discards, ; comments), as jepsen_amd/edn.py reads it.
// character classes: 1 whitespace (commas included), 2 token delimiter
struct EdnClasses {
    uint8_t c[256] = {};
    constexpr EdnClasses() {
        for (unsigned char w : {' ', ',', '\n', '\t', '\r', '\f', '\v'}) c[w] = 3;
        for (unsigned char d : {'[', ']', '{', '}', '(', ')', '"', ';', '#'}) c[d] = 2;
    }
};
constexpr EdnClasses EDN_CLS;
inline bool edn_ws(unsigned char c) { return EDN_CLS.c[c] & 1; }
inline bool edn_delim(unsigned char c) { return EDN_CLS.c[c] != 0; }

struct EdnParser {
    const char *s, *p, *e;
    Arena &A;
    IoErr err;
    int depth = 0;

    EdnParser(const char *base, const char *b, const char *end, Arena &a) : s(base), p(b), e(end), A(a) {}

    bool fail(const char *m) {
        if (err.code == JH_OK) { err.code = JH_EINVAL; err.msg = m; err.at = (size_t)(p - s); }
        return false;
    }
    void skip_ws() {
        for (;;) {
            while (p < e && edn_ws((unsigned char)*p)) p++;
            if (p < e && *p == ';') { while (p < e && *p != '\n') p++; continue; }
            break;
        }
    }
    std::string_view token() {
        const char *b = p;
        while (p < e && !edn_delim((unsigned char)*p)) p++;
        return std::string_view(b, (size_t)(p - b));
    }
    static void put_utf8(std::string &o, uint32_t cp) {
        if (cp < 0x80) o.push_back((char)cp);
        else if (cp < 0x800) { o.push_back((char)(0xC0 | (cp >> 6))); o.push_back((char)(0x80 | (cp & 63))); }
        else if (cp < 0x10000) {
            o.push_back((char)(0xE0 | (cp >> 12))); o.push_back((char)(0x80 | ((cp >> 6) & 63)));
            o.push_back((char)(0x80 | (cp & 63)));
        } else {
            o.push_back((char)(0xF0 | (cp >> 18))); o.push_back((char)(0x80 | ((cp >> 12) & 63)));
            o.push_back((char)(0x80 | ((cp >> 6) & 63))); o.push_back((char)(0x80 | (cp & 63)));
        }
    }
    static int hexv(char c) {
        if (c >= '0' && c <= '9') return c - '0';
        if (c >= 'a' && c <= 'f') return c - 'a' + 10;
        if (c >= 'A' && c <= 'F') return c - 'A' + 10;
        return -1;
    }
    bool string_(uint32_t &out) {
        p++;                                        // opening quote
        const char *b = p;
        bool esc = false;
        while (p < e && *p != '"') { if (*p == '\\') { esc = true; p++; } p++; }
        if (p >= e) return fail("unterminated string");
        if (!esc) { out = A.srctext(V_STR, b, (size_t)(p - b)); p++; return true; }
        std::string o;
        for (const char *q = b; q < p; q++) {
            if (*q != '\\') { o.push_back(*q); continue; }
            char c = *++q;
            if (c == 'u' && p - q > 4) {
                int h0 = hexv(q[1]), h1 = hexv(q[2]), h2 = hexv(q[3]), h3 = hexv(q[4]);
                if (h0 >= 0 && h1 >= 0 && h2 >= 0 && h3 >= 0) {
                    put_utf8(o, (uint32_t)(h0 << 12 | h1 << 8 | h2 << 4 | h3));
                    q += 4;
                    continue;
                }
            }
            switch (c) {
            case 'n': o.push_back('\n'); break;
            case 't': o.push_back('\t'); break;
            case 'r': o.push_back('\r'); break;
            case 'b': o.push_back('\b'); break;
            case 'f': o.push_back('\f'); break;
            default: o.push_back(c);
            }
        }
        p++;
        out = A.text(V_STR, o.data(), o.size());
        return true;
    }
    bool char_(uint32_t &out) {
        p++;                                        // backslash
        if (p >= e) return fail("bad character literal");
        static const struct { const char *n; char c; } named[] = {
            {"newline", '\n'}, {"space", ' '}, {"tab", '\t'}, {"return", '\r'}, {"formfeed", '\f'}, {"backspace", '\b'}};
        for (auto &nm : named) {
            size_t l = strlen(nm.n);
            if ((size_t)(e - p) >= l && memcmp(p, nm.n, l) == 0) { p += l; out = A.text(V_STR, &nm.c, 1); return true; }
        }
        if (*p == 'u' && e - p >= 5 && hexv(p[1]) >= 0 && hexv(p[2]) >= 0 && hexv(p[3]) >= 0 && hexv(p[4]) >= 0) {
            std::string o;
            put_utf8(o, (uint32_t)(hexv(p[1]) << 12 | hexv(p[2]) << 8 | hexv(p[3]) << 4 | hexv(p[4])));
            p += 5;
            out = A.text(V_STR, o.data(), o.size());
            return true;
        }
        // one code point
        const char *b = p++;
        while (p < e && ((unsigned char)*p & 0xC0) == 0x80) p++;
        out = A.text(V_STR, b, (size_t)(p - b));
        return true;
    }
    static bool all_digits(std::string_view t) {
        if (t.empty()) return false;
        for (char c : t) if (c < '0' || c > '9') return false;
        return true;
    }
    // edn.py's number regex: [+-]?\d+(?:/\d+|\.\d*(?:[eE][+-]?\d+)?M?|[eE][+-]?\d+M?|N|M)?
    bool number_(std::string_view t, uint32_t &out) {
        size_t i = 0;
        if (t[i] == '+' || t[i] == '-') i++;
        size_t d0 = i;
        while (i < t.size() && t[i] >= '0' && t[i] <= '9') i++;
        if (i == d0) return false;
        std::string_view ip = t.substr(0, i), rest = t.substr(i);
        // a decimal integer (optional sign, digits) checked against the int64 range
        auto checked = [&](std::string_view digits, bool neg, int64_t &v) -> bool {
            uint64_t u = 0;
            for (char c : digits) {
                const uint64_t d = (uint64_t)(c - '0');
                if (u > (UINT64_MAX - d) / 10) return false;
                u = u * 10 + d;
            }
            if (u > (neg ? (uint64_t)INT64_MAX + 1 : (uint64_t)INT64_MAX)) return false;
            v = neg ? (int64_t)(0 - u) : (int64_t)u;
            return true;
        };
        if (rest.empty() || rest == "N") {
            int64_t v = 0;
            if (!checked(ip.substr(d0), ip[0] == '-', v)) return fail("integer out of the int64 range");
            out = A.leaf(V_INT, v);
            return true;
        }
        if (rest[0] == '/') {
            if (!all_digits(rest.substr(1))) return false;
            // both parts through the integer path's checked accumulator (ADVICE
            // r2: strtoll saturated silently, and gcd of -LLONG_MIN is undefined)
            int64_t a = 0, b = 0;
            if (!checked(ip.substr(d0), ip[0] == '-', a) || !checked(rest.substr(1), false, b) ||
                a == INT64_MIN)
                return fail("ratio part out of the int64 range");
            if (b == 0) return fail("ratio with zero denominator");
            const int64_t g = std::gcd(a < 0 ? -a : a, b);
            if (g > 1) { a /= g; b /= g; }
            std::string r = std::to_string(a) + "/" + std::to_string(b);
            out = A.text(V_RATIO, r.data(), r.size());
            return true;
        }
        std::string_view f = rest;
        if (f.back() == 'M') f.remove_suffix(1);
        bool ok = false;
        if (f.empty()) ok = rest == "M";
        else if (f[0] == '.') {
            size_t j = 1;
            while (j < f.size() && f[j] >= '0' && f[j] <= '9') j++;
            if (j == f.size()) ok = true;
            else if (f[j] == 'e' || f[j] == 'E') {
                j++;
                if (j < f.size() && (f[j] == '+' || f[j] == '-')) j++;
                ok = j < f.size() && all_digits(f.substr(j));
            }
        } else if (f[0] == 'e' || f[0] == 'E') {
            size_t j = 1;
            if (j < f.size() && (f[j] == '+' || f[j] == '-')) j++;
            ok = j < f.size() && all_digits(f.substr(j)) && rest.substr(rest.size() - 1) != "N";
        }
        if (!ok) return false;
        std::string z(t.substr(0, t.size() - (t.back() == 'M' ? 1 : 0)));
        out = A.leaf(V_FLOAT, 0, strtod(z.c_str(), nullptr));
        return true;
    }
    // skips one form without building it (values of op-map keys nobody reads)
    bool skip_form() {
        skip_ws();
        if (p >= e) return fail("unexpected end of EDN input");
        int d = 0;
        do {
            if (d > 0) {
                skip_ws();
                if (p >= e) return fail("unterminated collection");
            }
            const char c = *p;
            if (c == '"') {
                p++;
                while (p < e && *p != '"') { if (*p == '\\') p++; p++; }
                if (p >= e) return fail("unterminated string");
                p++;
            } else if (c == '\\') {
                p += 2;
                while (p < e && !edn_delim((unsigned char)*p)) p++;
            } else if (c == '{' || c == '[' || c == '(') { d++; p++; }
            else if (c == '}' || c == ']' || c == ')') {
                if (d == 0) return fail("unexpected closing delimiter");
                d--; p++;
            } else if (c == '#') {
                p++;
                if (p < e && *p == '{') { d++; p++; }
                else if (p < e && *p == '_') {               // #_ discard: then the form itself
                    p++;
                    if (!skip_form()) return false;
                    if (d == 0) return skip_form();
                    continue;
                } else {                                     // a tag: its form follows
                    token();
                    if (!skip_form()) return false;
                    if (d == 0) return true;
                    continue;
                }
            } else {
                if (token().empty()) return fail("unreadable EDN");
                if (d == 0) return true;
                continue;
            }
        } while (d > 0);
        return true;
    }
    // a top-level op map: keyword keys matched in place, only the fields the
    // encoder reads are built, the others skipped
    template <class F>
    bool op_map(F &&field) {
        p++;                                            // '{'
        for (;;) {
            skip_ws();
            if (p >= e) return fail("unterminated collection");
            if (*p == '}') { p++; return true; }
            if (*p == '#' && p + 1 < e && p[1] == '_') { p += 2; if (!skip_form()) return false; continue; }
            std::string_view key;
            if (*p == ':') { p++; key = token(); }
            else {
                uint32_t k;
                if (!form(k)) return false;
                if (A.v[k].k == V_STR) key = A.sv(k);
            }
            skip_ws();
            if (p < e && *p == '#' && p + 1 < e && p[1] == '_') { p += 2; if (!skip_form()) return false; skip_ws(); }
            if (p >= e || *p == '}') return fail("map with an odd number of forms");
            if (field(key)) {
                uint32_t v;
                if (!form(v)) return false;
                field(key, v);
            } else if (!skip_form()) return false;
        }
    }
    bool seq_(char close, size_t &base) {
        base = A.stk.size();
        for (;;) {
            skip_ws();
            if (p >= e) return fail("unterminated collection");
            if (*p == close) { p++; return true; }
            if (*p == ']' || *p == '}' || *p == ')') return fail("mismatched closing delimiter");
            if (*p == '#' && p + 1 < e && p[1] == '_') {
                p += 2;
                uint32_t d;
                if (!form(d)) return false;
                A.v.pop_back();                       // discarded (its kids stay in the arena)
                continue;
            }
            uint32_t c;
            if (!form(c)) return false;
            A.stk.push_back(c);
        }
    }
    bool form(uint32_t &out) {
        skip_ws();
        if (p >= e) return fail("unexpected end of EDN input");
        if (++depth > 512) return fail("EDN nested too deeply");
        bool ok = form1(out);
        depth--;
        return ok;
    }
    bool form1(uint32_t &out) {
        const char c = *p;
        size_t base;
        switch (c) {
        case '{':
            p++;
            if (!seq_('}', base)) return false;
            if ((A.stk.size() - base) % 2) return fail("map with an odd number of forms");
            out = A.coll(V_MAP, base);
            return true;
        case '[': case '(':
            p++;
            if (!seq_(c == '[' ? ']' : ')', base)) return false;
            out = A.coll(V_VEC, base);
            return true;
        case '"': return string_(out);
        case '\\': return char_(out);
        case ']': case '}': case ')': return fail("unexpected closing delimiter");
        case '#': {
            if (p + 1 >= e) return fail("dangling #");
            if (p[1] == '{') {
                p += 2;
                if (!seq_('}', base)) return false;
                out = A.coll(V_SET, base);
                return true;
            }
            if (p[1] == '_') {
                p += 2;
                uint32_t d;
                if (!form(d)) return false;
                return form(out);
            }
            p++;
            std::string_view tag = token();
            if (tag.empty()) return fail("bad # dispatch");
            uint32_t f;
            if (!form(f)) return false;
            if ((tag == "inst" || tag == "uuid") && A.v[f].k == V_STR) { out = f; return true; }
            if (A.v[f].k == V_MAP) { out = f; return true; }        // a record literal: its map
            uint32_t toff = (uint32_t)A.txt.size();
            A.txt.append(tag);
            size_t b2 = A.stk.size();
            A.stk.push_back(f);
            out = A.coll(V_TAG, b2, toff, (uint32_t)tag.size());
            return true;
        }
        default: break;
        }
        {
            // fast path: a plain decimal integer followed by a delimiter
            const char *q = p;
            const bool neg = *q == '-';
            if (neg || *q == '+') q++;
            const char *d0 = q;
            uint64_t u = 0;
            while (q < e && *q >= '0' && *q <= '9' && q - d0 < 18) u = u * 10 + (uint64_t)(*q++ - '0');
            if (q > d0 && (q == e || edn_delim((unsigned char)*q))) {
                p = q;
                out = A.leaf(V_INT, neg ? -(int64_t)u : (int64_t)u);
                return true;
            }
        }
        std::string_view t = token();
        if (t.empty()) return fail("unreadable EDN");
        if ((t[0] >= '0' && t[0] <= '9') || ((t[0] == '+' || t[0] == '-') && t.size() > 1 && t[1] >= '0' && t[1] <= '9')) {
            if (number_(t, out)) return true;
            if (err.code) return false;
        }
        if (t == "nil") { out = A.leaf(V_NIL); return true; }
        if (t == "true") { out = A.leaf(V_TRUE); return true; }
        if (t == "false") { out = A.leaf(V_FALSE); return true; }
        if (t[0] == ':') { out = A.srctext(V_KW, t.data() + 1, t.size() - 1); return true; }
        out = A.srctext(V_SYM, t.data(), t.size());
        return true;
    }
};

// ---------------------------------------------------------------------------
// rows: history.encode's two passes over op maps (history.py:104-208)
enum { F_READ = JH_F_READ, F_CAS = JH_F_CAS, F_DRAIN = JH_F_DRAIN };

int known_f(std::string_view n) {
    if (n == "read") return JH_F_READ;
    if (n == "write") return JH_F_WRITE;
    if (n == "cas") return JH_F_CAS;
    if (n == "add") return JH_F_ADD;
    if (n == "enqueue") return JH_F_ENQUEUE;
    if (n == "dequeue") return JH_F_DEQUEUE;
    if (n == "drain") return JH_F_DRAIN;
    return -1;
}

struct Rows {
    std::vector<int64_t> proc, type, f, key, val, val2, time, aux;
    LocalTable procs, fs, keys, vals;
    bool ints_only = true;
    int64_t coll_row = -1;      // first row whose non-read collection value needs interning
    IoErr err;
    size_t end = 0;             // byte offset after the last form parsed
    void clear() {
        proc.clear(); type.clear(); f.clear(); key.clear(); val.clear(); val2.clear(); time.clear(); aux.clear();
        procs = LocalTable(); fs = LocalTable(); keys = LocalTable(); vals = LocalTable();
        ints_only = true; coll_row = -1; err = IoErr(); end = 0;
    }
};

struct Encoder {
    bool independent, intern;   // intern: pass 2, every value through the value table
    Arena &A;
    Rows &R;

    bool fail(const char *m, size_t at) {
        if (R.err.code == JH_OK) { R.err.code = JH_EINVAL; R.err.msg = m; R.err.at = at; }
        return false;
    }
    int64_t scalar(uint32_t x) {
        if (A.v[x].k == V_NIL) return JH_NIL;
        if (A.v[x].k == V_INT) return (int64_t)R.vals.get_int(A.v[x].i);
        std::string id = value_ident(A, x);
        std::string tx = id.substr(1);
        return (int64_t)R.vals.get(std::move(id), tx);
    }
    // element order of a set :read (history.py: sorted() when it can)
    void sorted_elems(uint32_t v, std::vector<uint32_t> &el) {
        const Val &e = A.v[v];
        el.clear();
        for (uint32_t j = 0; j < e.n; j++) el.push_back(A.kid(v, j));
        if (e.k != V_SET) return;
        bool num = true, str = true;
        for (uint32_t x : el) {
            uint8_t k = A.v[x].k;
            num &= k == V_INT || k == V_FLOAT || k == V_TRUE || k == V_FALSE;
            str &= k == V_STR || k == V_KW || k == V_SYM;
        }
        auto nv = [&](uint32_t x) -> long double {
            const Val &q = A.v[x];
            return q.k == V_INT ? (long double)q.i : q.k == V_FLOAT ? (long double)q.d : q.k == V_TRUE ? 1 : 0;
        };
        if (num) std::stable_sort(el.begin(), el.end(), [&](uint32_t a, uint32_t b) {
            const Val &x = A.v[a], &y = A.v[b];
            if (x.k == V_INT && y.k == V_INT) return x.i < y.i;
            return nv(a) < nv(b);
        });
        else if (str) std::stable_sort(el.begin(), el.end(), [&](uint32_t a, uint32_t b) { return A.sv(a) < A.sv(b); });
    }
    // the op map's fields (index into A.v, -1 = absent); a later duplicate key wins
    struct Fields { int64_t p = -1, t = -1, f = -1, v = -1, tm = -1; };
    static bool field(Fields &F, std::string_view n, int64_t val) {
        switch (n.size()) {
        case 1: if (n[0] == 'f') { F.f = val; return true; } break;
        case 4:
            if (n == "type") { F.t = val; return true; }
            if (n == "time") { F.tm = val; return true; }
            break;
        case 5: if (n == "value") { F.v = val; return true; } break;
        case 7: if (n == "process") { F.p = val; return true; } break;
        }
        return false;
    }
    bool row(uint32_t m, size_t at) {
        if (A.v[m].k != V_MAP) return fail("a history entry is not a map", at);
        const Val &mv = A.v[m];
        Fields F;
        for (uint32_t j = 0; j + 1 < mv.n; j += 2) {
            uint32_t k = A.kid(m, j);
            if (A.v[k].k != V_KW && A.v[k].k != V_STR) continue;
            field(F, A.sv(k), A.kid(m, j + 1));
        }
        return row(F, at);
    }
    bool row(const Fields &F, size_t at) {
        const int64_t p_x = F.p, t_x = F.t, f_x = F.f, v_x = F.v, tm_x = F.tm;
        // :type
        int typ = -1;
        if (t_x >= 0 && (A.v[t_x].k == V_KW || A.v[t_x].k == V_STR)) {
            std::string_view t = A.sv((uint32_t)t_x);
            typ = t == "invoke" ? JH_TYPE_INVOKE : t == "ok" ? JH_TYPE_OK : t == "fail" ? JH_TYPE_FAIL : t == "info" ? JH_TYPE_INFO : -1;
        }
        if (typ < 0) return fail("unknown :type", at);
        // :process (>= 0 integer: itself; else interned, -(1 + local id) until merged)
        int64_t proc;
        bool int_proc = false;
        if (p_x >= 0 && A.v[p_x].k == V_INT && A.v[p_x].i >= 0) { proc = A.v[p_x].i; int_proc = true; }
        else {
            std::string id, tx;
            if (p_x < 0) { id = "nnil"; tx = "nil"; }
            else { id = name_ident(A, (uint32_t)p_x); tx = name_text(A, (uint32_t)p_x); }
            proc = -1 - (int64_t)R.procs.get(std::move(id), tx);
            int_proc = p_x >= 0 && (A.v[p_x].k == V_INT || A.v[p_x].k == V_TRUE || A.v[p_x].k == V_FALSE);
        }
        // :f
        int64_t fc;
        {
            int kf = -1;
            if (f_x >= 0 && (A.v[f_x].k == V_KW || A.v[f_x].k == V_STR)) kf = known_f(A.sv((uint32_t)f_x));
            if (kf >= 0) fc = kf;
            else {
                std::string id, tx;
                if (f_x < 0) { id = "nnil"; tx = "nil"; }
                else { id = name_ident(A, (uint32_t)f_x); tx = name_text(A, (uint32_t)f_x); }
                fc = JH_F_FIRST_INTERNED_ + (int64_t)R.fs.get(std::move(id), tx);
            }
        }
        // :value, unwrapping an independent tuple
        int64_t v = v_x, keyid = -1;
        if (independent && int_proc && v >= 0 && A.v[v].k == V_VEC && A.v[v].n == 2) {
            uint32_t kx = A.kid((uint32_t)v, 0);
            if (A.v[kx].k == V_INT) keyid = (int64_t)R.keys.get_int(A.v[kx].i);
            else {
                std::string tx;
                canon(A, kx, tx);
                keyid = (int64_t)R.keys.get(name_ident(A, kx), tx);
            }
            v = A.kid((uint32_t)v, 1);
        }
        int64_t val = JH_NIL, val2 = JH_NIL;
        const bool isf_cas = fc < 16 && fc == F_CAS;
        const bool isf_rd = fc < 16 && (fc == F_READ || fc == F_DRAIN);
        if (v >= 0 && A.v[v].k != V_NIL) {
            const Val &vv = A.v[v];
            if (isf_cas && vv.k == V_VEC && vv.n == 2) {
                for (int j = 0; j < 2; j++) {
                    uint32_t x = A.kid((uint32_t)v, j);
                    int64_t o = JH_NIL;
                    if (intern) o = scalar(x);
                    else if (A.v[x].k == V_INT) {
                        if (A.v[x].i == JH_NIL) return fail("value collides with the nil sentinel", at);
                        o = A.v[x].i;
                    } else if (A.v[x].k != V_NIL) R.ints_only = false;
                    (j ? val2 : val) = o;
                }
            } else if (vv.k == V_VEC || vv.k == V_SET) {
                if (!intern)
                    for (uint32_t j = 0; j < vv.n; j++)
                        if (A.v[A.kid((uint32_t)v, j)].k != V_INT) { R.ints_only = false; break; }
                if (isf_rd) {
                    thread_local std::vector<uint32_t> el;
                    sorted_elems((uint32_t)v, el);
                    val = (int64_t)R.aux.size();
                    val2 = (int64_t)el.size();
                    for (uint32_t x : el) {
                        if (intern) R.aux.push_back(scalar(x));
                        else {
                            if (A.v[x].k == V_INT && A.v[x].i == JH_NIL) return fail("value collides with the nil sentinel", at);
                            R.aux.push_back(A.v[x].k == V_INT ? A.v[x].i : 0);
                        }
                    }
                } else if (intern) val = scalar((uint32_t)v);
                else if (R.coll_row < 0) R.coll_row = (int64_t)R.proc.size();
            } else if (intern) val = scalar((uint32_t)v);
            else if (vv.k == V_INT) {
                if (vv.i == JH_NIL) return fail("value collides with the nil sentinel", at);
                val = vv.i;
            } else R.ints_only = false;
        }
        R.proc.push_back(proc);
        R.type.push_back(typ);
        R.f.push_back(fc);
        R.key.push_back(keyid);
        R.val.push_back(val);
        R.val2.push_back(val2);
        R.time.push_back(tm_x >= 0 && A.v[tm_x].k == V_INT ? A.v[tm_x].i : JH_NIL);
        return true;
    }
    static constexpr int64_t JH_F_FIRST_INTERNED_ = 16;
};

// one EDN chunk: every form that starts in [b, lim) (the last may run past lim)
void parse_edn_chunk(const char *base, const char *b, const char *lim, const char *end, bool independent,
                     bool intern, Rows &R) {
    R.clear();
    {
        // rows are >= ~40 bytes: reserve once (untouched pages cost nothing)
        const size_t est = (size_t)(lim - b) / 40 + 16;
        for (auto *v : {&R.proc, &R.type, &R.f, &R.key, &R.val, &R.val2, &R.time}) v->reserve(est);
    }
    Arena A;
    EdnParser P(base, b, end, A);
    Encoder E{independent, intern, A, R};
    for (;;) {
        P.skip_ws();
        if (P.p >= lim || P.p >= end) break;
        A.reset();
        size_t at = (size_t)(P.p - base);
        if (*P.p == '{') {
            Encoder::Fields F;
            auto fld = [&](std::string_view k, int64_t v = -2) -> bool {
                if (v == -2) return k == "f" || k == "type" || k == "time" || k == "value" || k == "process";
                return Encoder::field(F, k, v);
            };
            if (!P.op_map(fld)) { R.err = P.err; break; }
            if (!E.row(F, at)) break;
            continue;
        }
        uint32_t m;
        if (!P.form(m)) { R.err = P.err; break; }
        if (A.v[m].k == V_VEC && P.p >= end && b == base && R.proc.empty()) {
            // a whole history as one vector literal read by one chunk
            std::vector<uint32_t> kids;
            for (uint32_t j = 0; j < A.v[m].n; j++) kids.push_back(A.kid(m, j));
            for (uint32_t k : kids) if (!E.row(k, at)) break;
            break;
        }
        if (!E.row(m, at)) break;
    }
    R.end = (size_t)(P.p - base);
}

// ---------------------------------------------------------------------------
// fressian (org.fressian codes; clojure.data.fressian + store.clj handlers)
struct FrParser {
    const uint8_t *s, *p, *e;
    Arena &A;
    Arena C;                         // cache entries (persist across ops)
    std::vector<uint32_t> pcache;    // priority cache -> node in C
    struct St { std::string tag; int64_t n; };
    std::vector<St> scache;
    IoErr err;
    int depth = 0;

    FrParser(const uint8_t *b, const uint8_t *end, Arena &a) : s(b), p(b), e(end), A(a) {}
    bool fail(const char *m) {
        if (err.code == JH_OK) { err.code = JH_EINVAL; err.msg = m; err.at = (size_t)(p - s); }
        return false;
    }
    bool need(size_t n) { return (size_t)(e - p) >= n ? true : fail("truncated fressian input"); }
    uint64_t raw(int n) {
        uint64_t v = 0;
        for (int i = 0; i < n; i++) v = v << 8 | *p++;
        return v;
    }
    bool int_code(int c, int64_t &v) {
        if (c == 0xFF) { v = -1; return true; }
        if (c <= 0x3F) { v = c; return true; }
        auto packed = [&](int zero, int nb) -> bool {
            if (!need((size_t)nb)) return false;
            v = (int64_t)((uint64_t)(int64_t)(c - zero) << (8 * nb)) | (int64_t)raw(nb);
            return true;
        };
        if (c >= 0x40 && c <= 0x5F) return packed(0x50, 1);
        if (c >= 0x60 && c <= 0x6F) return packed(0x68, 2);
        if (c >= 0x70 && c <= 0x73) return packed(0x72, 3);
        if (c >= 0x74 && c <= 0x77) return packed(0x76, 4);
        if (c >= 0x78 && c <= 0x7B) return packed(0x7A, 5);
        if (c >= 0x7C && c <= 0x7F) return packed(0x7E, 6);
        if (c == 0xF8) { if (!need(8)) return false; v = (int64_t)raw(8); return true; }
        return fail("expected a fressian int");
    }
    bool read_int(int64_t &v) {
        if (!need(1)) return false;
        return int_code(*p++, v);
    }
    // fressian strings are Java chars, 1-3 bytes each (surrogates apart); to UTF-8
    void jstr(const uint8_t *b, size_t n, std::string &o) {
        std::vector<uint32_t> u;
        for (size_t i = 0; i < n;) {
            uint8_t c = b[i];
            if (c < 0x80) { u.push_back(c); i++; }
            else if ((c >> 5) == 6 && i + 1 < n) { u.push_back((uint32_t)(c & 0x1F) << 6 | (b[i + 1] & 0x3F)); i += 2; }
            else if (i + 2 < n) {
                u.push_back((uint32_t)(c & 0x0F) << 12 | (uint32_t)(b[i + 1] & 0x3F) << 6 | (b[i + 2] & 0x3F));
                i += 3;
            } else break;
        }
        for (size_t i = 0; i < u.size(); i++) {
            uint32_t cp = u[i];
            if (cp >= 0xD800 && cp < 0xDC00 && i + 1 < u.size() && u[i + 1] >= 0xDC00 && u[i + 1] < 0xE000)
                cp = 0x10000 + ((cp - 0xD800) << 10) + (u[++i] - 0xDC00);
            EdnParser::put_utf8(o, cp);
        }
    }
    bool string_body(int c, std::string &o) {
        // STRING_PACKED 0xDA-0xE1, STRING 0xE3 len, STRING_CHUNK 0xE2 len ... then more
        for (;;) {
            int64_t n;
            bool chunk = false;
            if (c >= 0xDA && c <= 0xE1) n = c - 0xDA;
            else if (c == 0xE3 || c == 0xE2) { if (!read_int(n)) return false; chunk = c == 0xE2; }
            else return fail("expected a fressian string");
            if (n < 0 || !need((size_t)n)) return fail("bad fressian string length");
            jstr(p, (size_t)n, o);
            p += n;
            if (!chunk) return true;
            if (!need(1)) return false;
            c = *p++;
        }
    }
    bool bytes_body(int c, std::string &o) {
        for (;;) {
            int64_t n;
            bool chunk = false;
            if (c >= 0xD0 && c <= 0xD7) n = c - 0xD0;
            else if (c == 0xD9 || c == 0xD8) { if (!read_int(n)) return false; chunk = c == 0xD8; }
            else return fail("expected fressian bytes");
            if (n < 0 || !need((size_t)n)) return fail("bad fressian bytes length");
            o.append((const char *)p, (size_t)n);
            p += n;
            if (!chunk) return true;
            if (!need(1)) return false;
            c = *p++;
        }
    }
    // a list's elements pushed onto A.stk
    bool list_items(int c) {
        int64_t n = -1;
        if (c >= 0xE4 && c <= 0xEB) n = c - 0xE4;
        else if (c == 0xEC) { if (!read_int(n)) return false; }
        else if (c == 0xED || c == 0xEE) {
            for (;;) {
                if (p >= e) { if (c == 0xEE) return true; return fail("unterminated fressian list"); }
                if (*p == 0xFD) { p++; return true; }
                uint32_t x;
                if (!object(x)) return false;
                A.stk.push_back(x);
            }
        } else return fail("expected a fressian list");
        if (n < 0) return fail("negative list length");
        for (int64_t i = 0; i < n; i++) {
            uint32_t x;
            if (!object(x)) return false;
            A.stk.push_back(x);
        }
        return true;
    }
    bool list_object(size_t &base) {
        base = A.stk.size();
        if (!need(1)) return false;
        int c = *p++;
        if (c >= 0xE4 && c <= 0xEE && c != 0xE4 - 1) {
            if (c <= 0xEE) return list_items(c);
        }
        // anything else: one object that must be a vector
        p--;
        uint32_t x;
        if (!object(x)) return false;
        if (A.v[x].k != V_VEC && A.v[x].k != V_SET) return fail("expected a list");
        for (uint32_t j = 0; j < A.v[x].n; j++) A.stk.push_back(A.kid(x, j));
        return true;
    }
    uint32_t named(uint8_t k, uint32_t ns, uint32_t nm) {
        std::string t;
        if (A.v[ns].k == V_STR) { t += A.sv(ns); t.push_back('/'); }
        if (A.v[nm].k == V_STR) t += A.sv(nm);
        return A.text(k, t.data(), t.size());
    }
    bool structure(const St &st, uint32_t &out) {
        const std::string &tag = st.tag;
        const int64_t n = st.n;
        size_t base = A.stk.size();
        auto fields = [&]() -> bool {
            for (int64_t i = 0; i < n; i++) {
                uint32_t x;
                if (!object(x)) return false;
                A.stk.push_back(x);
            }
            return true;
        };
        if ((tag == "key" || tag == "sym") && n == 2) {
            if (!fields()) return false;
            uint32_t ns = A.stk[base], nm = A.stk[base + 1];
            A.stk.resize(base);
            out = named(tag == "key" ? V_KW : V_SYM, ns, nm);
            return true;
        }
        if ((tag == "map" || tag == "set" || tag == "vec" || tag == "list") && n == 1) {
            size_t b2;
            if (!list_object(b2)) return false;
            if (tag == "map" && (A.stk.size() - b2) % 2) return fail("map with an odd number of forms");
            out = A.coll(tag == "map" ? V_MAP : tag == "set" ? V_SET : V_VEC, b2);
            return true;
        }
        if (!fields()) return false;
        if (tag == "persistent-hash-set" || tag == "persistent-sorted-set") { out = A.coll(V_SET, base); return true; }
        if (tag == "map-entry" && n == 2) { out = A.coll(V_VEC, base); return true; }
        if ((tag == "atom" || tag == "instant" || tag == "date-time" || tag == "inst" || tag == "uri") && n == 1) {
            out = A.stk[base]; A.stk.resize(base); return true;
        }
        if (tag == "record" && n == 2 && A.v[A.stk[base + 1]].k == V_MAP) {
            out = A.stk[base + 1]; A.stk.resize(base); return true;
        }
        if (tag == "char" && n == 1 && A.v[A.stk[base]].k == V_INT) {
            std::string o;
            EdnParser::put_utf8(o, (uint32_t)A.v[A.stk[base]].i);
            A.stk.resize(base);
            out = A.text(V_STR, o.data(), o.size());
            return true;
        }
        uint32_t toff = (uint32_t)A.txt.size();
        A.txt.append(tag);
        out = A.coll(V_TAG, base, toff, (uint32_t)tag.size());
        return true;
    }
    bool object(uint32_t &out) {
        if (++depth > 512) return fail("fressian nested too deeply");
        bool ok = object1(out);
        depth--;
        return ok;
    }
    bool object1(uint32_t &out) {
        for (;;) {
            if (!need(1)) return false;
            const int c = *p++;
            if (c <= 0x7F || c == 0xFF || c == 0xF8) {
                int64_t v;
                if (!int_code(c, v)) return false;
                out = A.leaf(V_INT, v);
                return true;
            }
            if (c >= 0x80 && c <= 0x9F) return cache_get((int64_t)(c - 0x80), out);
            if (c >= 0xA0 && c <= 0xAF) {
                if ((size_t)(c - 0xA0) >= scache.size()) return fail("struct cache miss");
                St st = scache[c - 0xA0];
                return structure(st, out);
            }
            if ((c >= 0xDA && c <= 0xE3)) {
                std::string o;
                if (!string_body(c, o)) return false;
                out = A.text(V_STR, o.data(), o.size());
                return true;
            }
            if (c >= 0xD0 && c <= 0xD9) {
                std::string o;
                if (!bytes_body(c, o)) return false;
                std::string t = "#bytes \"";
                static const char hx[] = "0123456789abcdef";
                for (unsigned char b : o) { t.push_back(hx[b >> 4]); t.push_back(hx[b & 15]); }
                t.push_back('"');
                out = A.text(V_OPAQUE, t.data(), t.size());
                return true;
            }
            if (c >= 0xE4 && c <= 0xEE && c != 0xEF) {
                size_t base = A.stk.size();
                if (!list_items(c)) return false;
                out = A.coll(V_VEC, base);
                return true;
            }
            switch (c) {
            case 0xB0: case 0xB3: case 0xB1: case 0xB4: case 0xB2: case 0xB5: {
                int64_t n;
                if (!read_int(n) || n < 0) return fail("bad fressian array");
                size_t base = A.stk.size();
                for (int64_t i = 0; i < n; i++) {
                    uint32_t x;
                    if (c == 0xB1) { if (!need(8)) return false; uint64_t r = raw(8); double d; memcpy(&d, &r, 8); x = A.leaf(V_FLOAT, 0, d); }
                    else if (c == 0xB4) { if (!need(4)) return false; uint32_t r = (uint32_t)raw(4); float f; memcpy(&f, &r, 4); x = A.leaf(V_FLOAT, 0, f); }
                    else if (c == 0xB0 || c == 0xB3) { int64_t v; if (!read_int(v)) return false; x = A.leaf(V_INT, v); }
                    else if (!object(x)) return false;
                    A.stk.push_back(x);
                }
                out = A.coll(V_VEC, base);
                return true;
            }
            case 0xC0: case 0xC1: {
                size_t base;
                if (!list_object(base)) return false;
                if (c == 0xC0 && (A.stk.size() - base) % 2) return fail("map with an odd number of forms");
                out = A.coll(c == 0xC0 ? V_MAP : V_SET, base);
                return true;
            }
            case 0xC9: case 0xCA: {
                uint32_t ns, nm;
                if (!object(ns) || !object(nm)) return false;
                out = named(c == 0xCA ? V_KW : V_SYM, ns, nm);
                return true;
            }
            case 0xC3: case 0xC4: case 0xC5: case 0xC8: {
                uint32_t x;
                if (!object(x)) return false;
                if (c == 0xC5 || c == 0xC3 || A.v[x].k != V_INT) { out = x; return true; }
                std::string t = "#inst " + std::to_string(A.v[x].i);
                out = A.text(V_OPAQUE, t.data(), t.size());
                return true;
            }
            case 0xC6: case 0xC7: {
                uint32_t b;
                if (!object(b)) return false;
                int64_t scale = 0;
                if (c == 0xC7 && !read_int(scale)) return false;
                std::string_view hexs = A.sv(b);                       // #bytes "...."
                std::string h(hexs.substr(8, hexs.size() >= 9 ? hexs.size() - 9 : 0));
                if (h.size() > 16) return fail("bigint out of the int64 range");
                uint64_t u = h.empty() ? 0 : strtoull(h.c_str(), nullptr, 16);
                int bits = (int)h.size() * 4;
                int64_t v = bits == 0 ? 0 : bits >= 64 ? (int64_t)u : (int64_t)(u << (64 - bits)) >> (64 - bits);
                if (c == 0xC6) out = A.leaf(V_INT, v);
                else out = A.leaf(V_FLOAT, 0, (double)v * std::pow(10.0, (double)-scale));
                return true;
            }
            case 0xCC: { int64_t i; if (!read_int(i)) return false; return cache_get(i, out); }
            case 0xCD: {
                uint32_t x;
                if (!object(x)) return false;
                pcache.push_back(copy_tree(A, x, C));
                out = x;
                return true;
            }
            case 0xCE: {
                uint32_t x;
                if (!object(x)) return false;
                pcache.push_back(copy_tree(A, x, C));
                continue;                                 // precache: read the next object
            }
            case 0xCF: return fail("fressian footer inside a value");
            case 0xEF: {
                uint32_t t;
                if (!object(t)) return false;
                int64_t n;
                if (!read_int(n) || n < 0) return fail("bad struct type");
                St st{std::string(A.v[t].k == V_STR || A.v[t].k == V_SYM || A.v[t].k == V_KW ? A.sv(t) : std::string_view("?")), n};
                scache.push_back(st);
                return structure(st, out);
            }
            case 0xF0: {
                int64_t i;
                if (!read_int(i)) return false;
                if (i < 0 || (size_t)i >= scache.size()) return fail("struct cache miss");
                St st = scache[(size_t)i];
                return structure(st, out);
            }
            case 0xF1: { uint32_t m; if (!object(m)) return false; continue; }   // meta, then the object
            case 0xF5: out = A.leaf(V_TRUE); return true;
            case 0xF6: out = A.leaf(V_FALSE); return true;
            case 0xF7: out = A.leaf(V_NIL); return true;
            case 0xF9: { if (!need(4)) return false; uint32_t r = (uint32_t)raw(4); float f; memcpy(&f, &r, 4); out = A.leaf(V_FLOAT, 0, f); return true; }
            case 0xFA: { if (!need(8)) return false; uint64_t r = raw(8); double d; memcpy(&d, &r, 8); out = A.leaf(V_FLOAT, 0, d); return true; }
            case 0xFB: out = A.leaf(V_FLOAT, 0, 0.0); return true;
            case 0xFC: out = A.leaf(V_FLOAT, 0, 1.0); return true;
            case 0xFE: pcache.clear(); scache.clear(); continue;                 // reset caches
            default: return fail("unknown fressian code");
            }
        }
    }
    bool cache_get(int64_t i, uint32_t &out) {
        if (i < 0 || (size_t)i >= pcache.size()) return fail("priority cache miss");
        out = copy_tree(C, pcache[(size_t)i], A);
        return true;
    }
};

// test.fressian (the test map; :history streamed) or a bare history vector
void parse_fressian(const uint8_t *b, size_t n, bool independent, bool intern, Rows &R) {
    R.clear();
    Arena A;
    FrParser P(b, b + n, A);
    Encoder E{independent, intern, A, R};
    auto fail = [&]() { if (R.err.code == JH_OK) R.err = P.err; };
    // the ops of a history list, one at a time (arena reset per op)
    auto stream_ops = [&](int c) -> bool {
        int64_t cnt = -1;
        bool open = false;
        if (c >= 0xE4 && c <= 0xEB) cnt = c - 0xE4;
        else if (c == 0xEC) { if (!P.read_int(cnt)) return false; }
        else if (c == 0xED || c == 0xEE) open = true;
        else return P.fail("expected the history list");
        for (int64_t i = 0; open || i < cnt; i++) {
            if (open) {
                if (P.p >= P.e) { if (c == 0xEE) break; return P.fail("unterminated history list"); }
                if (*P.p == 0xFD) { P.p++; break; }
            }
            A.reset();
            size_t at = (size_t)(P.p - b);
            uint32_t m;
            if (!P.object(m)) return false;
            if (!E.row(m, at)) return false;
        }
        return true;
    };
    // peeks through a "vec"/"list" struct wrapper to the list code
    auto history_value = [&]() -> bool {
        for (;;) {
            if (!P.need(1)) return false;
            int c = *P.p;
            if (c >= 0xE4 && c <= 0xEE) { P.p++; return stream_ops(c); }
            const FrParser::St *st = nullptr;
            const uint8_t *save = P.p;
            if (c >= 0xA0 && c <= 0xAF && (size_t)(c - 0xA0) < P.scache.size()) { st = &P.scache[c - 0xA0]; P.p++; }
            else if (c == 0xEF) {
                P.p++;
                uint32_t t;
                if (!P.object(t)) return false;
                int64_t nf;
                if (!P.read_int(nf)) return false;
                P.scache.push_back({std::string(A.v[t].k == V_STR ? A.sv(t) : std::string_view("?")), nf});
                st = &P.scache.back();
            }
            if (st && (st->tag == "vec" || st->tag == "list") && st->n == 1) continue;
            if (st) P.p = save;          // not a wrapper: generic parse below (cache entry already made)
            if (st && c == 0xEF) { P.scache.pop_back(); }
            A.reset();
            uint32_t x;
            if (!P.object(x)) return false;
            if (A.v[x].k != V_VEC) return P.fail(":history is not a list");
            size_t at = (size_t)(P.p - b);
            std::vector<uint32_t> ops;
            for (uint32_t j = 0; j < A.v[x].n; j++) ops.push_back(A.kid(x, j));
            for (uint32_t o : ops) if (!E.row(o, at)) return false;
            return true;
        }
    };
    bool ok = true;
    if (!P.need(1)) { fail(); return; }
    int c0 = *P.p;
    if (c0 == 0xC0) {
        // {... :history [...] ...}: stream the map's list of k v
        P.p++;
        if (!P.need(1)) { fail(); return; }
        int lc = *P.p++;
        int64_t cnt = -1;
        bool open = false;
        if (lc >= 0xE4 && lc <= 0xEB) cnt = lc - 0xE4;
        else if (lc == 0xEC) ok = P.read_int(cnt);
        else if (lc == 0xED || lc == 0xEE) open = true;
        else ok = P.fail("expected the test map's entries");
        bool found = false;
        for (int64_t i = 0; ok && (open || i < cnt); i += 2) {
            if (open) {
                if (P.p >= P.e) break;
                if (*P.p == 0xFD) { P.p++; break; }
            }
            A.reset();
            uint32_t k;
            if (!(ok = P.object(k))) break;
            if (!found && (A.v[k].k == V_KW || A.v[k].k == V_STR) && A.sv(k) == "history") {
                found = true;
                ok = history_value();
            } else {
                A.reset();
                uint32_t v;
                ok = P.object(v);
            }
        }
        if (ok && !found) ok = P.fail("no :history in the fressian test map");
    } else if (c0 >= 0xE4 && c0 <= 0xEE) {
        P.p++;
        ok = stream_ops(c0);
    } else {
        ok = history_value();
    }
    if (!ok) fail();
    R.end = (size_t)(P.p - b);
}

}  // namespace

// ---------------------------------------------------------------------------
struct jh_ingest {
    std::vector<int64_t> proc, type, f, key, val, val2, time, aux;
    std::vector<std::string> tables[3];
    int interned = 0;
};

namespace {

void set_err(char *err, size_t errlen, const std::string &m) {
    if (err && errlen) { snprintf(err, errlen, "%s", m.c_str()); }
}

// merge local tables in chunk order -> global ids (first appearance order)
struct Merge {
    std::unordered_map<std::string, int64_t> ids;
    std::vector<std::string> text;
    std::vector<std::vector<int64_t>> remap;
};

void merge_table(std::vector<Rows> &rs, LocalTable Rows::*tbl, Merge &M, int64_t first, int64_t step) {
    M.remap.assign(rs.size(), {});
    for (size_t c = 0; c < rs.size(); c++) {
        LocalTable &L = rs[c].*tbl;
        auto &rm = M.remap[c];
        rm.resize(L.ident.size());
        for (size_t j = 0; j < L.ident.size(); j++) {
            auto it = M.ids.find(L.ident[j]);
            if (it == M.ids.end()) {
                int64_t id = first + step * (int64_t)M.text.size();
                it = M.ids.emplace(L.ident[j], id).first;
                M.text.push_back(L.text[j]);
            }
            rm[j] = it->second;
        }
    }
}

int run_chunks(const char *buf, size_t len, int format, bool independent, const jh_ingest_opts &o, bool intern,
               std::vector<Rows> &rs, IoErr &err) {
    const int threads = o.threads;
    if (format == JH_FMT_FRESSIAN) {
        rs.assign(1, Rows());
        parse_fressian((const uint8_t *)buf, len, independent, intern, rs[0]);
        if (rs[0].err.code) { err = rs[0].err; return err.code; }
        return JH_OK;
    }
    // EDN: strip a history vector literal's outer brackets
    const char *b = buf, *e = buf + len;
    {
        const char *q = b;
        while (q < e && (edn_ws((unsigned char)*q) || *q == ';')) {
            if (*q == ';') while (q < e && *q != '\n') q++;
            else q++;
        }
        if (q < e && *q == '[') {
            const char *z = e;
            while (z > q && edn_ws((unsigned char)z[-1])) z--;
            if (z > q + 1 && z[-1] == ']') {
                // only when the vector's elements are maps: [{...} {...}]
                const char *r = q + 1;
                while (r < z && edn_ws((unsigned char)*r)) r++;
                if (r == z - 1 || *r == '{' || *r == '#') { b = q + 1; e = z - 1; }
            }
        }
    }
    const size_t n = (size_t)(e - b);
    int T = threads > 0 ? threads : (int)std::max(1u, std::thread::hardware_concurrency());
    // chunks of >= 1 MiB (jh_ingest_opts.min_chunk: smaller, for the boundary tests)
    const size_t min_chunk = o.min_chunk > 0 ? (size_t)o.min_chunk : (size_t)1 << 20;
    T = (int)std::max<size_t>(1, std::min<size_t>((size_t)T, n / min_chunk + 1));
    std::vector<const char *> st(T + 1);
    st[0] = b;
    st[T] = e;
    for (int i = 1; i < T; i++) {
        const char *q = b + n / T * i;
        if (q < st[i - 1]) q = st[i - 1];
        while (q < e && *q != '\n') q++;
        st[i] = q < e ? q + 1 : e;
    }
    rs.assign(T, Rows());
    {
        std::vector<std::thread> th;
        for (int i = 0; i < T; i++)
            th.emplace_back([&, i]() {
                auto t0 = std::chrono::steady_clock::now();
                parse_edn_chunk(buf, st[i], st[i + 1], e, independent, intern, rs[i]);
                if (o.debug)
                    fprintf(stderr, "[jh-ingest] chunk %d: %zu bytes, %zu rows, %.3f s\n", i, (size_t)(st[i + 1] - st[i]),
                            rs[i].proc.size(), std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
            });
        for (auto &t : th) t.join();
    }
    // verify the speculative boundaries; re-parse the rest sequentially at the first miss
    for (int i = 0; i < T; i++) {
        if (rs[i].err.code) {
            if (i > 0 && rs[i - 1].end != (size_t)(st[i] - buf)) { /* started inside a form */ }
            else { err = rs[i].err; return err.code; }
        }
        if (i + 1 < T) {
            // the next chunk's start must be where this chunk stopped (after whitespace)
            const char *q = buf + rs[i].end;
            while (q < st[i + 1] && (edn_ws((unsigned char)*q))) q++;
            if (q == st[i + 1] && !rs[i + 1].err.code) continue;
            if (rs[i].err.code) { err = rs[i].err; return err.code; }
            if (o.debug)
                fprintf(stderr, "[jh-ingest] chunk %d ends at %zu, chunk %d starts at %zu (err %d: %s): sequential re-parse\n", i,
                        rs[i].end, i + 1, (size_t)(st[i + 1] - buf), rs[i + 1].err.code, rs[i + 1].err.msg.c_str());
            Rows tail;
            parse_edn_chunk(buf, buf + rs[i].end, e, e, independent, intern, tail);
            rs.resize(i + 2);
            rs[i + 1] = std::move(tail);
            if (rs[i + 1].err.code) { err = rs[i + 1].err; return err.code; }
            break;
        }
    }
    return JH_OK;
}

int ingest(const char *buf, size_t len, int format, int independent, const jh_ingest_opts &o, jh_ingest **out,
           char *err, size_t errlen) {
    if (!out) { set_err(err, errlen, "null out"); return JH_EINVAL; }
    *out = nullptr;
    if (format == JH_FMT_AUTO) {
        size_t i = 0;
        while (i < len && edn_ws((unsigned char)buf[i])) i++;
        unsigned char c = i < len ? (unsigned char)buf[i] : '{';
        format = (c == '{' || c == '[' || c == '#' || c == ';' || c == '(') ? JH_FMT_EDN : JH_FMT_FRESSIAN;
        if (len == 0) format = JH_FMT_EDN;
    }
    if (format != JH_FMT_EDN && format != JH_FMT_FRESSIAN) { set_err(err, errlen, "unknown format"); return JH_EINVAL; }
    try {
        const bool dbg = o.debug != 0;
        auto now = []() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); };
        double t0 = now();
        std::vector<Rows> rs;
        IoErr e;
        int rc = run_chunks(buf, len, format, independent != 0, o, false, rs, e);
        bool ints_only = true;
        int64_t coll_row = -1, rowbase = 0;
        if (rc == JH_OK)
            for (auto &r : rs) {
                ints_only &= r.ints_only;
                if (coll_row < 0 && r.coll_row >= 0) coll_row = rowbase + r.coll_row;
                rowbase += (int64_t)r.proc.size();
            }
        if (rc == JH_OK && !ints_only) rc = run_chunks(buf, len, format, independent != 0, o, true, rs, e);
        if (rc != JH_OK) {
            char m[96];
            snprintf(m, sizeof m, "%s byte %zu: ", format == JH_FMT_EDN ? "EDN" : "fressian", e.at);
            set_err(err, errlen, m + e.msg);
            return rc;
        }
        if (ints_only && coll_row >= 0) {
            char m[128];
            snprintf(m, sizeof m, "row %lld: a collection :value on an op that is not a :read / :cas "
                     "(history.encode cannot take it as an integer)", (long long)coll_row);
            set_err(err, errlen, m);
            return JH_EUNSUPPORTED;
        }
        double t1 = now();
        auto *g = new jh_ingest();
        g->interned = ints_only ? 0 : 1;
        Merge mp, mf, mk, mv;
        mp.ids.emplace("snemesis", -1);
        mp.text.push_back("\"nemesis\"");
        merge_table(rs, &Rows::procs, mp, -1, -1);
        merge_table(rs, &Rows::fs, mf, 16, 1);
        merge_table(rs, &Rows::keys, mk, 0, 1);
        merge_table(rs, &Rows::vals, mv, 0, 1);
        size_t N = 0, NA = 0;
        std::vector<size_t> rb(rs.size()), ab(rs.size());
        for (size_t c = 0; c < rs.size(); c++) { rb[c] = N; ab[c] = NA; N += rs[c].proc.size(); NA += rs[c].aux.size(); }
        for (auto *v : {&g->proc, &g->type, &g->f, &g->key, &g->val, &g->val2, &g->time}) v->resize(N);
        g->aux.resize(NA ? NA : 1, 0);
        std::vector<std::thread> th;
        for (size_t c = 0; c < rs.size(); c++)
            th.emplace_back([&, c]() {
                Rows &r = rs[c];
                const size_t o = rb[c];
                const int64_t abase = (int64_t)ab[c];
                const bool rd_aux = true;
                for (size_t i = 0; i < r.proc.size(); i++) {
                    int64_t p = r.proc[i];
                    g->proc[o + i] = p >= 0 ? p : mp.remap[c][(size_t)(-1 - p)];
                    g->type[o + i] = r.type[i];
                    int64_t f = r.f[i];
                    g->f[o + i] = f < 16 ? f : mf.remap[c][(size_t)(f - 16)];
                    g->key[o + i] = r.key[i] < 0 ? -1 : mk.remap[c][(size_t)r.key[i]];
                    g->time[o + i] = r.time[i];
                    const bool aux_row = rd_aux && f < 16 && (f == JH_F_READ || f == JH_F_DRAIN) && r.val2[i] != JH_NIL &&
                                         !(f == JH_F_CAS);
                    int64_t v = r.val[i], v2 = r.val2[i];
                    if (aux_row && v != JH_NIL) { v += abase; }
                    else if (g->interned) {
                        if (v != JH_NIL) v = mv.remap[c][(size_t)v];
                        if (v2 != JH_NIL) v2 = mv.remap[c][(size_t)v2];
                    }
                    g->val[o + i] = v;
                    g->val2[o + i] = v2;
                }
                for (size_t j = 0; j < r.aux.size(); j++) {
                    int64_t x = r.aux[j];
                    g->aux[ab[c] + j] = g->interned && x != JH_NIL ? mv.remap[c][(size_t)x] : x;
                }
            });
        for (auto &t : th) t.join();
        if (dbg)
            fprintf(stderr, "[jh-ingest] %zu chunk(s), parse %.3f s (interned pass: %d), merge %.3f s\n", rs.size(), t1 - t0,
                    ints_only ? 0 : 1, now() - t1);
        g->tables[JH_TBL_KEYS] = std::move(mk.text);
        g->tables[JH_TBL_F] = std::move(mf.text);
        g->tables[JH_TBL_VALUES] = std::move(mv.text);
        *out = g;
        return JH_OK;
    } catch (const std::bad_alloc &) {
        set_err(err, errlen, "out of host memory");
        return JH_ENOMEM;
    } catch (const std::exception &x) {
        set_err(err, errlen, x.what());
        return JH_EINVAL;
    }
}

jh_ingest_opts plain_opts(int threads) {
    jh_ingest_opts o;
    memset(&o, 0, sizeof o);
    o.threads = threads;
    return o;
}

}  // namespace

extern "C" {

int jh_ingest_buffer_opts(const char *buf, size_t len, int format, int independent, const jh_ingest_opts *opts,
                          jh_ingest **out, char *err, size_t errlen) {
    if (!buf && len) { set_err(err, errlen, "null buffer"); return JH_EINVAL; }
    const jh_ingest_opts o = opts ? *opts : plain_opts(0);
    return ingest(buf ? buf : "", len, format, independent, o, out, err, errlen);
}

int jh_ingest_file_opts(const char *path, int format, int independent, const jh_ingest_opts *opts, jh_ingest **out,
                        char *err, size_t errlen) {
    if (!path) { set_err(err, errlen, "null path"); return JH_EINVAL; }
    const jh_ingest_opts o = opts ? *opts : plain_opts(0);
    int fd = open(path, O_RDONLY);
    if (fd < 0) { set_err(err, errlen, std::string("cannot open ") + path); return JH_EINVAL; }
    struct stat sb;
    if (fstat(fd, &sb) != 0) { close(fd); set_err(err, errlen, "cannot stat the history file"); return JH_EINVAL; }
    size_t len = (size_t)sb.st_size;
    if (len == 0) { close(fd); return ingest("", 0, format, independent, o, out, err, errlen); }
    void *m = mmap(nullptr, len, PROT_READ, MAP_PRIVATE, fd, 0);
    close(fd);
    if (m == MAP_FAILED) { set_err(err, errlen, "cannot map the history file"); return JH_EINVAL; }
    madvise(m, len, MADV_SEQUENTIAL);
    int rc = ingest((const char *)m, len, format, independent, o, out, err, errlen);
    munmap(m, len);
    return rc;
}

int jh_ingest_buffer(const char *buf, size_t len, int format, int independent, int threads, jh_ingest **out,
                     char *err, size_t errlen) {
    const jh_ingest_opts o = plain_opts(threads);
    return jh_ingest_buffer_opts(buf, len, format, independent, &o, out, err, errlen);
}

int jh_ingest_file(const char *path, int format, int independent, int threads, jh_ingest **out, char *err,
                   size_t errlen) {
    const jh_ingest_opts o = plain_opts(threads);
    return jh_ingest_file_opts(path, format, independent, &o, out, err, errlen);
}

void jh_ingest_history(const jh_ingest *g, jh_history *h) {
    if (!g || !h) return;
    memset(h, 0, sizeof *h);
    h->n = (int64_t)g->proc.size();
    h->process = g->proc.data();
    h->type = g->type.data();
    h->f = g->f.data();
    h->key = g->key.data();
    h->value = g->val.data();
    h->value2 = g->val2.data();
    h->n_keys = (int64_t)g->tables[JH_TBL_KEYS].size();
    h->aux = g->aux.data();
    h->n_aux = (int64_t)g->aux.size();
    h->on_device = 0;
}

const int64_t *jh_ingest_time(const jh_ingest *g) { return g ? g->time.data() : nullptr; }

int jh_ingest_values_interned(const jh_ingest *g) { return g ? g->interned : 0; }

int64_t jh_ingest_table_size(const jh_ingest *g, int table) {
    if (!g || table < 0 || table > 2) return -1;
    return (int64_t)g->tables[table].size();
}

int64_t jh_ingest_table_entry(const jh_ingest *g, int table, int64_t i, char *buf, size_t cap) {
    if (!g || table < 0 || table > 2 || i < 0 || (size_t)i >= g->tables[table].size()) return -1;
    const std::string &s = g->tables[table][(size_t)i];
    if (buf && cap) {
        size_t n = std::min(cap - 1, s.size());
        memcpy(buf, s.data(), n);
        buf[n] = 0;
    }
    return (int64_t)s.size();
}

void jh_ingest_free(jh_ingest *g) { delete g; }

}  // extern "C"
