// meshio.cpp -- native mesh loaders (OBJ, binary and ASCII STL) behind include/sdfgen_meshio.h.
//
// The callers on the input side of the hot path: the reference parses
// OBJ and ASCII STL with one std::istringstream per line (common/mesh_io_obj.cpp:52-131,
// common/mesh_io_stl.cpp:179-303) and reads binary STL with two seeks per facet (:98-173).
// Here the whole file is read at once and text formats are parsed in parallel chunks split at
// line boundaries, with the reference's line grammar and its results bit for bit:
//   * numbers: `istream >> float` is a correctly rounded decimal conversion of the longest
//     numeric prefix (libstdc++ num_get + strtof in the C locale); std::from_chars is the same
//     conversion, locale-free.  num_get accepts a leading '+', no "inf"/"nan" (with or without
//     a sign) and no hex, and FAILS on an exponent marker with no digits ("1e", "2E+"): it
//     consumes the 'e' and the sign, and strtof then does not use the whole token.
//   * OBJ faces: v, v/vt, v/vt/vn, v//vn -- the index before the first '/' through std::stoi
//     semantics (leading whitespace, optional sign, digits; an invalid token is an error), then
//     1-based -> 0-based as uint32 (wrapping), fan triangulation (mesh_io_obj.cpp:115-121).
//   * bounds: meshio::update_minmax per accepted vertex (common/mesh_io.h:101-108: std::min and
//     std::max applied independently; the non-template overload wins over util.h's else-if one),
//     computed in one ordered pass.
//   * a binary STL with 0 facets loads as an empty mesh (mesh_io_stl.cpp:140-172 returns true).
// All of this is pinned against the reference loaders compiled from their sources
// (tests/test_meshio_ref.py, oracle/mesh_ref_shim.cpp).
#include "sdfgen_meshio.h"

#include <algorithm>
#include <cctype>
#include <charconv>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <string>
#include <thread>
#include <vector>

struct sdfgen_mesh {
    std::vector<float> xyz;        // nvert x 3
    std::vector<uint32_t> tri;     // ntri x 3
    float bounds[6];               // min xyz, max xyz
    int format = 0;
};

namespace {

int fail(char *errbuf, size_t errlen, int code, const char *fmt, ...)
{
    if (errbuf && errlen) {
        va_list ap;
        va_start(ap, fmt);
        vsnprintf(errbuf, errlen, fmt, ap);
        va_end(ap);
    }
    return code;
}

bool read_file(const char *path, std::vector<char> &buf)
{
    FILE *f = fopen(path, "rb");
    if (!f) return false;
    if (fseek(f, 0, SEEK_END) != 0) { fclose(f); return false; }
    const long n = ftell(f);
    if (n < 0 || fseek(f, 0, SEEK_SET) != 0) { fclose(f); return false; }
    buf.resize((size_t)n + 1);
    const size_t got = n ? fread(buf.data(), 1, (size_t)n, f) : 0;
    fclose(f);
    if (got != (size_t)n) return false;
    buf[(size_t)n] = '\0';
    buf.resize((size_t)n);
    return true;
}

inline bool is_ws(char c) { return c == ' ' || c == '\t' || c == '\n' || c == '\r' || c == '\v' || c == '\f'; }

// `is >> float` from p (whitespace skipped first): false when no number can be read.
inline bool parse_float(const char *&p, const char *end, float &v)
{
    while (p < end && is_ws(*p)) ++p;
    if (p >= end) return false;
    const char *q = p;
    if (*q == '+') ++q;   // num_get takes a leading '+', from_chars does not
    const char *m = q < end && (*q == '+' || *q == '-') ? q + 1 : q;
    if (m < end && (*m == 'i' || *m == 'I' || *m == 'n' || *m == 'N')) return false;   // no [+-]inf / nan
    if (q + 1 < end && q[0] == '0' && (q[1] == 'x' || q[1] == 'X')) {   // num_get reads "0", stops at 'x'
        v = 0.0f;
        if (*p == '-') v = -0.0f;
        p = q + 1;
        return true;
    }
    if (*p == '+' && q < end && *q == '-') return false;
    const char *s = *p == '+' ? q : p;
    auto r = std::from_chars(s, end, v, std::chars_format::general);
    if (r.ec == std::errc::invalid_argument) return false;
    if (r.ec == std::errc::result_out_of_range) {
        // num_get (strtof) keeps an underflowed value (a denormal or +-0) and fails only on
        // overflow; from_chars reports both as out of range: redo this token with strtof.
        char tok[128];
        const size_t len = std::min<size_t>((size_t)(r.ptr - s), sizeof(tok) - 1);
        memcpy(tok, s, len);
        tok[len] = '\0';
        const float w = strtof(tok, nullptr);
        if (w == std::numeric_limits<float>::infinity() || w == -std::numeric_limits<float>::infinity()) return false;
        v = w;
    }
    if (r.ptr < end && (*r.ptr == 'e' || *r.ptr == 'E')) {
        // from_chars stopped at an exponent marker: either the token already had its exponent
        // ("1e2e3": num_get stops there too) or the marker has no digits, which num_get consumes
        // and then fails on.
        bool had_exp = false;
        for (const char *c = s; c < r.ptr; ++c) had_exp |= *c == 'e' || *c == 'E';
        if (!had_exp) return false;
    }
    p = r.ptr;
    return true;
}

// std::stoi on the token [b, e): leading whitespace, sign, digits; throws (here: false) if none.
inline bool stoi_prefix(const char *b, const char *e, int32_t &out)
{
    while (b < e && is_ws(*b)) ++b;
    bool neg = false;
    if (b < e && (*b == '+' || *b == '-')) neg = *b++ == '-';
    if (b >= e || *b < '0' || *b > '9') return false;
    long long v = 0;
    while (b < e && *b >= '0' && *b <= '9') {
        v = v * 10 + (*b++ - '0');
        if (v > (long long)std::numeric_limits<int32_t>::max() + 1) return false;   // out_of_range
    }
    v = neg ? -v : v;
    if (v > std::numeric_limits<int32_t>::max() || v < std::numeric_limits<int32_t>::min()) return false;
    out = (int32_t)v;
    return true;
}

// Chunk boundaries at line starts: T pieces of [0, n).
std::vector<size_t> split_lines(const std::vector<char> &buf, int T)
{
    const size_t n = buf.size();
    std::vector<size_t> cut{0};
    for (int t = 1; t < T; ++t) {
        size_t c = std::max(cut.back(), n * (size_t)t / (size_t)T);
        while (c < n && c > 0 && buf[c - 1] != '\n') ++c;
        cut.push_back(c);
    }
    cut.push_back(n);
    return cut;
}

int n_threads(size_t bytes)
{
    const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
    const size_t by_size = bytes / (4u << 20) + 1;   // ~4 MB of text per thread at least
    return (int)std::min<size_t>({(size_t)hw, (size_t)16, by_size});
}

struct ObjPart {
    std::vector<float> xyz;
    std::vector<uint32_t> tri;
    bool bad = false;
    size_t bad_line = 0;
};

void parse_obj_chunk(const char *b, const char *e, ObjPart &out)
{
    std::vector<int32_t> idx;
    for (const char *ls = b; ls < e;) {
        const char *le = static_cast<const char *>(memchr(ls, '\n', (size_t)(e - ls)));
        if (!le) le = e;
        const size_t len = (size_t)(le - ls);
        if (len > 0) {
            const char c0 = ls[0], c1 = len > 1 ? ls[1] : '\0';
            if (c0 == 'v' && (c1 == ' ' || c1 == '\t')) {   // "vn" / "vt" and others are skipped
                const char *p = ls + 1;
                float x, y, z;
                if (parse_float(p, le, x) && parse_float(p, le, y) && parse_float(p, le, z)) {
                    out.xyz.push_back(x);
                    out.xyz.push_back(y);
                    out.xyz.push_back(z);
                }   // else: the reference warns and skips the line
            } else if (c0 == 'f' && (c1 == ' ' || c1 == '\t')) {
                idx.clear();
                const char *p = ls + 1;
                while (true) {
                    while (p < le && is_ws(*p)) ++p;
                    if (p >= le) break;
                    const char *t = p;
                    while (p < le && !is_ws(*p)) ++p;
                    const char *slash = static_cast<const char *>(memchr(t, '/', (size_t)(p - t)));
                    int32_t v;
                    if (!stoi_prefix(t, slash ? slash : p, v)) {
                        out.bad = true;   // std::stoi throws: the reference's load fails
                        return;
                    }
                    idx.push_back(v);
                }
                if (idx.size() >= 3)
                    for (size_t q = 1; q + 1 < idx.size(); ++q) {
                        out.tri.push_back((uint32_t)(idx[0] - 1));
                        out.tri.push_back((uint32_t)(idx[q] - 1));
                        out.tri.push_back((uint32_t)(idx[q + 1] - 1));
                    }
            }
        }
        ls = le + 1;
    }
}

// meshio::update_minmax (common/mesh_io.h:101-108) over the vertices in file order:
// min = std::min(min, x) = (x < min) ? x : min, max = std::max(max, x) = (max < x) ? x : max.
void update_bounds(const std::vector<float> &xyz, float b[6])
{
    for (int c = 0; c < 3; ++c) {
        b[c] = std::numeric_limits<float>::max();
        b[3 + c] = std::numeric_limits<float>::lowest();
    }
    const size_t n = xyz.size() / 3;
    for (size_t v = 0; v < n; ++v)
        for (int c = 0; c < 3; ++c) {
            const float x = xyz[3 * v + c];
            if (x < b[c]) b[c] = x;
            if (b[3 + c] < x) b[3 + c] = x;
        }
}

int load_obj(const std::vector<char> &buf, sdfgen_mesh &m, char *errbuf, size_t errlen)
{
    const int T = n_threads(buf.size());
    const std::vector<size_t> cut = split_lines(buf, T);
    std::vector<ObjPart> part(T);
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t)
        th.emplace_back([&, t] { parse_obj_chunk(buf.data() + cut[t], buf.data() + cut[t + 1], part[t]); });
    for (auto &x : th) x.join();
    size_t nv = 0, nt = 0;
    for (auto &p : part) {
        if (p.bad) return fail(errbuf, errlen, SDFGEN_MESH_EFORMAT, "invalid face index in OBJ file");
        nv += p.xyz.size();
        nt += p.tri.size();
    }
    m.xyz.reserve(nv);
    m.tri.reserve(nt);
    for (auto &p : part) {
        m.xyz.insert(m.xyz.end(), p.xyz.begin(), p.xyz.end());
        m.tri.insert(m.tri.end(), p.tri.begin(), p.tri.end());
    }
    if (m.xyz.empty()) return fail(errbuf, errlen, SDFGEN_MESH_EFORMAT, "No vertices found in OBJ file");
    if (m.tri.empty()) return fail(errbuf, errlen, SDFGEN_MESH_EFORMAT, "No faces found in OBJ file");
    return 0;
}

// Binary STL (mesh_io_stl.cpp:98-173): 80-byte header, uint32 count, 50-byte facets
// (normal, 3 vertices, attribute); vertices 3t, 3t+1, 3t+2 per facet, no de-duplication.
int load_binary_stl(const std::vector<char> &buf, sdfgen_mesh &m, char *errbuf, size_t errlen)
{
    if (buf.size() < 84) return fail(errbuf, errlen, SDFGEN_MESH_EFORMAT, "truncated binary STL");
    uint32_t n;
    memcpy(&n, buf.data() + 80, 4);
    if (buf.size() < 84 + (size_t)n * 50) return fail(errbuf, errlen, SDFGEN_MESH_EFORMAT, "truncated binary STL");
    m.xyz.resize((size_t)n * 9);
    m.tri.resize((size_t)n * 3);
    for (size_t t = 0; t < n; ++t) {
        memcpy(&m.xyz[9 * t], buf.data() + 84 + 50 * t + 12, 36);
        m.tri[3 * t] = (uint32_t)(3 * t);
        m.tri[3 * t + 1] = (uint32_t)(3 * t + 1);
        m.tri[3 * t + 2] = (uint32_t)(3 * t + 2);
    }
    return 0;   // n == 0: an empty mesh, as the reference returns (no "no faces" check for binary)
}

inline bool starts_ci(const char *p, const char *e, const char *kw)
{
    for (; *kw; ++kw, ++p)
        if (p >= e || std::tolower((unsigned char)*p) != *kw) return false;
    return true;
}

// ASCII STL (mesh_io_stl.cpp:179-303): keywords matched case-insensitively at the start of
// each whitespace-trimmed line, in the reference's order; vertex lines parsed as
// `keyword >> x >> y >> z`.  Two phases: line chunks are classified and their vertex numbers
// parsed in parallel (the cost: 3 correctly rounded floats per vertex line), then the state
// machine replays the line events in file order, so errors surface exactly where the
// sequential reference would stop.
enum : uint8_t { STL_SOLID, STL_ENDSOLID, STL_FACET, STL_ENDFACET, STL_LOOP, STL_ENDLOOP, STL_VERTEX, STL_BADVERTEX };

struct StlPart {
    std::vector<uint8_t> ev;   // one event per keyword line
    std::vector<float> xyz;    // the numbers of its STL_VERTEX events, in order
};

void parse_stl_chunk(const char *b, const char *e, StlPart &out)
{
    for (const char *ls = b; ls < e;) {
        const char *le = static_cast<const char *>(memchr(ls, '\n', (size_t)(e - ls)));
        if (!le) le = e;
        const char *p = ls;
        while (p < le && is_ws(*p)) ++p;
        if (p < le) {
            if (starts_ci(p, le, "solid")) out.ev.push_back(STL_SOLID);
            else if (starts_ci(p, le, "endsolid")) out.ev.push_back(STL_ENDSOLID);
            else if (starts_ci(p, le, "facet")) out.ev.push_back(STL_FACET);
            else if (starts_ci(p, le, "endfacet")) out.ev.push_back(STL_ENDFACET);
            else if (starts_ci(p, le, "outer loop")) out.ev.push_back(STL_LOOP);
            else if (starts_ci(p, le, "endloop")) out.ev.push_back(STL_ENDLOOP);
            else if (starts_ci(p, le, "vertex")) {
                const char *q = p;
                while (q < le && !is_ws(*q)) ++q;   // the keyword token
                float x, y, z;
                if (parse_float(q, le, x) && parse_float(q, le, y) && parse_float(q, le, z)) {
                    out.ev.push_back(STL_VERTEX);
                    out.xyz.push_back(x);
                    out.xyz.push_back(y);
                    out.xyz.push_back(z);
                } else {
                    out.ev.push_back(STL_BADVERTEX);
                }
            }
        }
        ls = le + 1;
    }
}

int load_ascii_stl(const std::vector<char> &buf, sdfgen_mesh &m, char *errbuf, size_t errlen)
{
    const int T = n_threads(buf.size());
    const std::vector<size_t> cut = split_lines(buf, T);
    std::vector<StlPart> part(T);
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t)
        th.emplace_back([&, t] { parse_stl_chunk(buf.data() + cut[t], buf.data() + cut[t + 1], part[t]); });
    for (auto &x : th) x.join();
    size_t nv = 0;
    for (auto &p : part) nv += p.xyz.size();
    m.xyz.reserve(nv);
    bool in_solid = false, in_facet = false, in_loop = false;
    int in_facet_n = 0;
    uint32_t start = 0;
    for (auto &p : part) {
        size_t vi = 0;
        for (const uint8_t ev : p.ev) {
            switch (ev) {
            case STL_SOLID: in_solid = true; break;
            case STL_ENDSOLID: in_solid = false; break;
            case STL_FACET:
                if (!in_solid) return fail(errbuf, errlen, SDFGEN_MESH_EFORMAT, "'facet' outside 'solid' block");
                in_facet = true;
                in_facet_n = 0;
                start = (uint32_t)(m.xyz.size() / 3);
                break;
            case STL_ENDFACET:
                if (in_facet_n != 3)
                    return fail(errbuf, errlen, SDFGEN_MESH_EFORMAT, "Facet has %d vertices (expected 3)", in_facet_n);
                in_facet = false;
                m.tri.push_back(start);
                m.tri.push_back(start + 1);
                m.tri.push_back(start + 2);
                break;
            case STL_LOOP: in_loop = true; break;
            case STL_ENDLOOP: in_loop = false; break;
            default:   // STL_VERTEX, STL_BADVERTEX
                if (!in_facet || !in_loop) return fail(errbuf, errlen, SDFGEN_MESH_EFORMAT, "'vertex' outside facet/loop");
                if (ev == STL_BADVERTEX) return fail(errbuf, errlen, SDFGEN_MESH_EFORMAT, "Failed to parse vertex");
                m.xyz.insert(m.xyz.end(), p.xyz.begin() + vi, p.xyz.begin() + vi + 3);
                vi += 3;
                ++in_facet_n;
                break;
            }
        }
    }
    if (m.xyz.empty()) return fail(errbuf, errlen, SDFGEN_MESH_EFORMAT, "No vertices found in ASCII STL file");
    if (m.tri.empty()) return fail(errbuf, errlen, SDFGEN_MESH_EFORMAT, "No faces found in ASCII STL file");
    return 0;
}

// Format detection, mesh_io_stl.cpp:42-92: no leading "solid" (case-insensitive) -> binary;
// with it, binary only if the file size matches the facet count exactly.
bool stl_is_binary(const std::vector<char> &buf)
{
    const size_t h = std::min<size_t>(buf.size(), 80);
    if (h >= 5 && starts_ci(buf.data(), buf.data() + h, "solid")) {
        if (buf.size() < 84) return false;
        uint32_t n;
        memcpy(&n, buf.data() + 80, 4);
        return (unsigned long long)buf.size() == 84ull + 50ull * n;
    }
    return true;
}

}  // namespace

extern "C" {

int sdfgen_mesh_load(const char *path, int format, sdfgen_mesh **out, char *errbuf, size_t errlen)
{
    if (errbuf && errlen) errbuf[0] = 0;
    if (!path || !out) return fail(errbuf, errlen, SDFGEN_MESH_EINVAL, "null pointer argument");
    *out = nullptr;
    std::vector<char> buf;
    if (!read_file(path, buf)) return fail(errbuf, errlen, SDFGEN_MESH_EIO, "Failed to load mesh: %s", path);
    if (format == SDFGEN_MESH_AUTO) {
        const std::string s(path);
        std::string ext = s.size() >= 4 ? s.substr(s.size() - 4) : "";
        std::transform(ext.begin(), ext.end(), ext.begin(), [](unsigned char c) { return (char)std::tolower(c); });
        if (ext == ".obj") format = SDFGEN_MESH_OBJ;
        else if (ext == ".stl") format = SDFGEN_MESH_STL;
        else return fail(errbuf, errlen, SDFGEN_MESH_EINVAL, "Failed to load mesh: %s (unsupported format)", path);
    }
    if (format == SDFGEN_MESH_STL) {
        if (buf.size() < 5) return fail(errbuf, errlen, SDFGEN_MESH_EFORMAT, "Failed to load mesh: %s", path);
        format = stl_is_binary(buf) ? SDFGEN_MESH_STL_BINARY : SDFGEN_MESH_STL_ASCII;
    }
    sdfgen_mesh *m = new sdfgen_mesh();
    int rc;
    if (format == SDFGEN_MESH_OBJ) rc = load_obj(buf, *m, errbuf, errlen);
    else if (format == SDFGEN_MESH_STL_BINARY) rc = load_binary_stl(buf, *m, errbuf, errlen);
    else if (format == SDFGEN_MESH_STL_ASCII) rc = load_ascii_stl(buf, *m, errbuf, errlen);
    else rc = fail(errbuf, errlen, SDFGEN_MESH_EINVAL, "unknown mesh format %d", format);
    if (rc) {
        delete m;
        return rc;
    }
    m->format = format;
    update_bounds(m->xyz, m->bounds);
    *out = m;
    return 0;
}

int sdfgen_mesh_info(const sdfgen_mesh *m, uint64_t *nvert, uint64_t *ntri, float bounds[6], int *format)
{
    if (!m) return SDFGEN_MESH_EINVAL;
    if (nvert) *nvert = m->xyz.size() / 3;
    if (ntri) *ntri = m->tri.size() / 3;
    if (bounds) memcpy(bounds, m->bounds, sizeof(m->bounds));
    if (format) *format = m->format;
    return 0;
}

int sdfgen_mesh_copy(const sdfgen_mesh *m, float *xyz, uint32_t *tri)
{
    if (!m) return SDFGEN_MESH_EINVAL;
    if (xyz && !m->xyz.empty()) memcpy(xyz, m->xyz.data(), m->xyz.size() * sizeof(float));
    if (tri && !m->tri.empty()) memcpy(tri, m->tri.data(), m->tri.size() * sizeof(uint32_t));
    return 0;
}

int sdfgen_mesh_free(sdfgen_mesh *m)
{
    delete m;
    return 0;
}

}  // extern "C"
