// pt_ingest.h — native OBJ reader with the reference's semantics
// (scene_reader.py:49-104 + vector.py:143-173), for large meshes (K5's
// 100k triangles) where the reference's per-line Python parse dominates
// setup.  Host code only; bound as pt_obj_load / pt_mesh_free.
//
// Semantics kept exactly:
//   * lines split like Python text-mode readlines (\n, \r\n, \r);
//   * remove_all_comments (scene_reader.py:29-46): leading spaces stripped,
//     '#' lines dropped, anything after '#' cut, '\t' -> ' ';
//   * tokens = split(' ') without empty tokens (scene_reader.py:11-26);
//   * `v x y z`: float() of each token; `f i j k ...`: int() indices, i < 0
//     counts back from the vertices read so far, else i - 1; more than three
//     indices are fan triangulated from the first (scene_reader.py:66-83);
//   * normal = normalize(cross(v2 - v1, v3 - v1)), area = |cross| / 2 with the
//     reference's operation order: V.__sub__ is a + (-b), size() =
//     sqrt(0 + c0**2 + c1**2 + c2**2) with Python's ** (C pow), normalize
//     multiplies by 1/size.
// Inputs the fast reader does not mirror byte for byte (hex or underscore
// numbers, `1/2/3` face tokens, faces with < 3 indices, out-of-range
// indices, vertices with other than 3 coordinates, a line of only spaces)
// return PT_EUNSUPPORTED: the Python reader then parses the file and raises
// exactly what the reference raises.
#pragma once
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <new>
#include <string>
#include <thread>
#include <vector>

namespace pt {

struct MeshOut {
    std::vector<double> vert;        // [n_vert][3]
    std::vector<int64_t> face;       // [n_tri][3] as Obj.faces holds them (before Python's wrap)
    std::vector<double> tri_v, tri_n, tri_area;
    std::vector<int64_t> skip_off, skip_len;   // raw lines of skipped commands
};

// Python float() on a token (ASCII decimal, inf, nan; surrounding whitespace
// allowed).  Returns false for what this reader does not mirror.
inline bool py_float(const char* b, const char* e, double* out) {
    while (b < e && (*b == '\v' || *b == '\f' || *b == '\r' || *b == ' ')) ++b;
    while (e > b && (e[-1] == '\v' || e[-1] == '\f' || e[-1] == '\r' || e[-1] == ' ')) --e;
    if (b == e || e - b > 64) return false;
    char buf[72];
    size_t n = 0;
    for (const char* p = b; p < e; ++p) {
        const char c = *p;
        const bool ok = (c >= '0' && c <= '9') || c == '.' || c == '+' || c == '-' || c == 'e' ||
                        c == 'E';
        if (!ok) {   // inf / nan spellings: leave to Python
            return false;
        }
        buf[n++] = c;
    }
    buf[n] = 0;
    char* end = nullptr;
    *out = strtod(buf, &end);
    return end == buf + n;
}

// Python int() on a token: [+-]digits only here.
inline bool py_int(const char* b, const char* e, int64_t* out) {
    while (b < e && (*b == '\v' || *b == '\f' || *b == '\r' || *b == ' ')) ++b;
    while (e > b && (e[-1] == '\v' || e[-1] == '\f' || e[-1] == '\r' || e[-1] == ' ')) --e;
    if (b == e) return false;
    bool neg = false;
    if (*b == '+' || *b == '-') { neg = (*b == '-'); ++b; }
    if (b == e || e - b > 18) return false;
    int64_t v = 0;
    for (const char* p = b; p < e; ++p) {
        if (*p < '0' || *p > '9') return false;
        v = v * 10 + (*p - '0');
    }
    *out = neg ? -v : v;
    return true;
}

// normal and area of one triangle, vector.py order of operations
inline void tri_normal_area(const double* a, const double* b, const double* c, double* n,
                            double* area) {
    const double u[3] = {(-a[0]) + b[0], (-a[1]) + b[1], (-a[2]) + b[2]};
    const double v[3] = {(-a[0]) + c[0], (-a[1]) + c[1], (-a[2]) + c[2]};
    const double x[3] = {u[1] * v[2] - u[2] * v[1], u[2] * v[0] - u[0] * v[2],
                         u[0] * v[1] - u[1] * v[0]};
    // Python's c ** 2 is libm pow(c, 2.0), which is not always the correctly
    // rounded c * c (glibc differs in ~1e-3 of cases): call pow itself,
    // through a volatile pointer so the compiler cannot fold it to c * c
    double (*volatile libm_pow)(double, double) = static_cast<double (*)(double, double)>(&::pow);
    double s = 0.0;
    for (int i = 0; i < 3; ++i) s = s + libm_pow(x[i], 2.0);
    const double size = sqrt(s);
    const double k = 1.0 / size;   // normalize: v * (1 / size); size 0 -> inf / nan, as Python
    for (int i = 0; i < 3; ++i) n[i] = x[i] * k;
    *area = size / 2;
}

enum : int { kIngestOk = 0, kIngestIo = 1, kIngestUnsupported = 2, kIngestDivZero = 3 };

// The parse runs in two parallel phases over chunks of whole lines (each
// chunk but the last ends just after a '\n', so no line and no "\r\n" is
// split), with the file order of everything that depends on it restored in
// between:
//   A (per chunk): lines -> vertex coordinates, face lines as raw index
//     tokens with the chunk-local vertex count at that line, skipped lines;
//     stops at the chunk's first malformed line;
//   (serial) vertex counts -> each chunk's first vertex number; all vertices
//     in file order;
//   C (per chunk): each face's indices resolved against the vertices read
//     before its line (Python's negative indexing), normals and areas; stops
//     at the chunk's first out-of-range index or zero area.
// The result is the first error in file order — the chunk-local errors of
// the first chunk that has one (C's precede A's: phase A stopped at its error
// line) — or the chunks' outputs concatenated: the serial reader's, bit for
// bit.  PT_INGEST_CHUNK (bytes, default 1 MiB) is the smallest chunk;
// threads: OMP_NUM_THREADS, else the machine's, at most 16.
struct ObjChunk {
    size_t off = 0;                       // chunk start in the file
    std::vector<double> vert;             // [n][3], chunk-local
    std::vector<int64_t> frec;            // per face line: line offset, local nv, n, n raw indices
    std::vector<int64_t> skip_off, skip_len;
    int err = kIngestOk;                  // phase A's first error
    bool non_ascii = false;               // a byte >= 0x80 or NUL anywhere in the chunk
    int64_t nv = 0;                       // vertices in the chunk
    // phase C
    std::vector<int64_t> face;
    std::vector<double> tri_v, tri_n, tri_area;
    int cerr = kIngestOk;
};

inline void parse_obj_chunk(const char* data, size_t size, bool last, ObjChunk* C) {
    unsigned char acc = 0, nul = 1;
    for (size_t i = 0; i < size; ++i) {
        acc |= (unsigned char)data[i];
        nul &= (unsigned char)(data[i] != 0);
    }
    if ((acc & 0x80u) || !nul) {   // non-ASCII: leave the file to Python's decoder
        C->non_ascii = true;
        return;
    }
    C->vert.reserve(size / 24);
    std::vector<std::pair<const char*, const char*>> tok;
    size_t pos = 0;
    while (pos < size) {
        // one physical line (universal newlines)
        size_t end = pos;
        while (end < size && data[end] != '\n' && data[end] != '\r') ++end;
        const size_t line_b = pos, line_e = end;
        size_t next = end;
        if (next < size) next += (data[next] == '\r' && next + 1 < size && data[next + 1] == '\n') ? 2 : 1;
        const bool had_newline = end < size || !last;
        pos = next;
        // remove_spaces_from_start: an all-space line without a newline walks
        // off the end (IndexError in the reference)
        size_t b = line_b;
        while (b < line_e && data[b] == ' ') ++b;
        if (b == line_e && !had_newline) { C->err = kIngestUnsupported; return; }
        if (b == line_e) continue;            // "\n" -> "" -> no tokens
        if (data[b] == '#') continue;
        size_t e = b;
        while (e < line_e && data[e] != '#') ++e;   // split('#')[0]
        // tokens: split on ' ' after '\t' -> ' '
        tok.clear();
        size_t i = b;
        while (i < e) {
            while (i < e && (data[i] == ' ' || data[i] == '\t')) ++i;
            const size_t s = i;
            while (i < e && data[i] != ' ' && data[i] != '\t') ++i;
            if (i > s) tok.emplace_back(data + s, data + i);
        }
        if (tok.empty()) continue;
        const size_t klen = (size_t)(tok[0].second - tok[0].first);
        if (klen == 1 && tok[0].first[0] == 'v') {
            if (tok.size() != 4) { C->err = kIngestUnsupported; return; }
            for (int c = 0; c < 3; ++c) {
                double x;
                if (!py_float(tok[1 + c].first, tok[1 + c].second, &x)) { C->err = kIngestUnsupported; return; }
                C->vert.push_back(x);
            }
            ++C->nv;
        } else if (klen == 1 && tok[0].first[0] == 'f') {
            if (tok.size() < 4) { C->err = kIngestUnsupported; return; }   // < 3 indices: IndexError
            C->frec.push_back((int64_t)line_b);
            C->frec.push_back(C->nv);
            C->frec.push_back((int64_t)tok.size() - 1);
            for (size_t t = 1; t < tok.size(); ++t) {
                int64_t v;
                if (!py_int(tok[t].first, tok[t].second, &v)) { C->err = kIngestUnsupported; return; }
                C->frec.push_back(v);
            }
        } else {
            C->skip_off.push_back((int64_t)(C->off + line_b));
            C->skip_len.push_back((int64_t)(line_e - line_b));
        }
    }
}

// phase C of one chunk: v0 = the chunk's first vertex number, V all vertices
inline void resolve_obj_chunk(ObjChunk* C, int64_t v0, const double* V) {
    std::vector<int64_t> raw, idx;
    size_t p = 0;
    while (p < C->frec.size()) {
        const int64_t n_vert = v0 + C->frec[p + 1];   // vertices read before this line
        const size_t n = (size_t)C->frec[p + 2];
        const int64_t* tk = &C->frec[p + 3];
        p += 3 + n;
        raw.clear();
        idx.clear();
        for (size_t t = 0; t < n; ++t) {
            const int64_t v = tk[t];
            const int64_t r = v < 0 ? n_vert + v : v - 1;   // Obj.faces holds this
            const int64_t k = r < 0 ? r + n_vert : r;       // Python negative indexing
            if (k < 0 || k >= n_vert) { C->cerr = kIngestUnsupported; return; }   // IndexError
            raw.push_back(r);
            idx.push_back(k);
        }
        for (size_t j = 1; j + 1 < idx.size(); ++j) {   // fan (a triangle when 3)
            const size_t q3[3] = {0, j, j + 1};
            double nr[3], area;
            tri_normal_area(V + 3 * idx[0], V + 3 * idx[j], V + 3 * idx[j + 1], nr, &area);
            if (!(area != 0.0)) { C->cerr = kIngestDivZero; return; }   // 1/0: ZeroDivisionError
            for (int q = 0; q < 3; ++q) {
                C->face.push_back(raw[q3[q]]);
                for (int c = 0; c < 3; ++c) C->tri_v.push_back(V[3 * idx[q3[q]] + c]);
                C->tri_n.push_back(nr[q]);
            }
            C->tri_area.push_back(area);
        }
    }
}

inline int ingest_threads() {
    const char* e = getenv("OMP_NUM_THREADS");
    int n = e ? atoi(e) : 0;
    if (n <= 0) n = (int)std::thread::hardware_concurrency();
    return n < 1 ? 1 : (n > 16 ? 16 : n);
}

// run f(i) for i < n on up to `threads` threads; a worker's bad_alloc is
// rethrown here
template <class F>
inline void ingest_parallel(int n, int threads, F f) {
    if (n <= 1 || threads <= 1) {
        for (int i = 0; i < n; ++i) f(i);
        return;
    }
    std::atomic<int> next{0};
    std::atomic<bool> oom{false};
    std::vector<std::thread> pool;
    const int nt = threads < n ? threads : n;
    for (int t = 0; t < nt; ++t)
        pool.emplace_back([&]() {
            for (int i; (i = next.fetch_add(1)) < n;) {
                try {
                    f(i);
                } catch (const std::bad_alloc&) {
                    oom = true;
                }
            }
        });
    for (auto& th : pool) th.join();
    if (oom) throw std::bad_alloc();
}

inline int parse_obj_text(const char* data, size_t size, MeshOut* M) {
    const char* ce = getenv("PT_INGEST_CHUNK");
    long long min_chunk = ce ? atoll(ce) : 0;
    if (min_chunk <= 0) min_chunk = 1 << 20;
    const int threads = ingest_threads();
    size_t want = size / (size_t)min_chunk;
    if (want < 1) want = 1;
    if (want > (size_t)threads * 4) want = (size_t)threads * 4;
    std::vector<size_t> cut{0};   // chunk boundaries: just after a '\n'
    for (size_t k = 1; k < want; ++k) {
        size_t p = size * k / want;
        if (p <= cut.back()) continue;
        while (p < size && data[p - 1] != '\n') ++p;
        if (p < size && p > cut.back()) cut.push_back(p);
    }
    cut.push_back(size);
    const int nc = (int)cut.size() - 1;
    std::vector<ObjChunk> ch((size_t)nc);
    ingest_parallel(nc, threads, [&](int i) {
        ch[(size_t)i].off = cut[(size_t)i];
        parse_obj_chunk(data + cut[(size_t)i], cut[(size_t)i + 1] - cut[(size_t)i], i == nc - 1, &ch[(size_t)i]);
    });
    for (const ObjChunk& C : ch)
        if (C.non_ascii) return kIngestUnsupported;
    // vertices in file order, up to the first malformed line
    std::vector<int64_t> v0((size_t)nc, 0);
    int64_t nv = 0;
    int stop = nc;   // chunks after the first phase-A error are not reached
    for (int i = 0; i < nc; ++i) {
        v0[(size_t)i] = nv;
        nv += ch[(size_t)i].nv;
        if (ch[(size_t)i].err != kIngestOk) { stop = i + 1; break; }
    }
    M->vert.reserve((size_t)nv * 3);
    for (int i = 0; i < stop; ++i)
        M->vert.insert(M->vert.end(), ch[(size_t)i].vert.begin(), ch[(size_t)i].vert.end());
    const double* V = M->vert.data();
    ingest_parallel(stop, threads, [&](int i) { resolve_obj_chunk(&ch[(size_t)i], v0[(size_t)i], V); });
    size_t nt = 0, ns = 0;
    for (int i = 0; i < stop; ++i) {
        const ObjChunk& C = ch[(size_t)i];
        if (C.cerr != kIngestOk) return C.cerr;   // before the chunk's phase-A error
        if (C.err != kIngestOk) return C.err;
        nt += C.tri_area.size();
        ns += C.skip_off.size();
    }
    M->face.reserve(nt * 3);
    M->tri_v.reserve(nt * 9);
    M->tri_n.reserve(nt * 3);
    M->tri_area.reserve(nt);
    M->skip_off.reserve(ns);
    M->skip_len.reserve(ns);
    for (int i = 0; i < stop; ++i) {
        const ObjChunk& C = ch[(size_t)i];
        M->face.insert(M->face.end(), C.face.begin(), C.face.end());
        M->tri_v.insert(M->tri_v.end(), C.tri_v.begin(), C.tri_v.end());
        M->tri_n.insert(M->tri_n.end(), C.tri_n.begin(), C.tri_n.end());
        M->tri_area.insert(M->tri_area.end(), C.tri_area.begin(), C.tri_area.end());
        M->skip_off.insert(M->skip_off.end(), C.skip_off.begin(), C.skip_off.end());
        M->skip_len.insert(M->skip_len.end(), C.skip_len.begin(), C.skip_len.end());
    }
    return kIngestOk;
}

inline int parse_obj_file(const char* path, MeshOut* M) {
    FILE* f = fopen(path, "rb");
    if (!f) return kIngestIo;
    std::string buf;
    if (fseek(f, 0, SEEK_END) == 0) {   // size the buffer once (a regular file)
        const long n = ftell(f);
        if (n > 0) buf.reserve((size_t)n);
        rewind(f);
    }
    char chunk[1 << 16];
    size_t got;
    while ((got = fread(chunk, 1, sizeof(chunk), f)) > 0) buf.append(chunk, got);
    const bool err = ferror(f) != 0;
    fclose(f);
    if (err) return kIngestIo;
    return parse_obj_text(buf.data(), buf.size(), M);   // (non-ASCII: kIngestUnsupported)
}

}  // namespace pt
