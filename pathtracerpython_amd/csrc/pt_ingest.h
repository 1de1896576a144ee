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

#include <string>
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

inline int parse_obj_text(const char* data, size_t size, MeshOut* M) {
    std::vector<std::pair<const char*, const char*>> tok;
    int64_t n_vert = 0;
    size_t pos = 0;
    while (pos < size) {
        // one physical line (universal newlines)
        size_t end = pos;
        while (end < size && data[end] != '\n' && data[end] != '\r') ++end;
        const size_t line_b = pos, line_e = end;
        size_t next = end;
        if (next < size) next += (data[next] == '\r' && next + 1 < size && data[next + 1] == '\n') ? 2 : 1;
        const bool had_newline = end < size;
        pos = next;
        // remove_spaces_from_start: an all-space line without a newline walks
        // off the end (IndexError in the reference)
        size_t b = line_b;
        while (b < line_e && data[b] == ' ') ++b;
        if (b == line_e && !had_newline) return kIngestUnsupported;
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
            if (tok.size() != 4) return kIngestUnsupported;
            for (int c = 0; c < 3; ++c) {
                double x;
                if (!py_float(tok[1 + c].first, tok[1 + c].second, &x)) return kIngestUnsupported;
                M->vert.push_back(x);
            }
            ++n_vert;
        } else if (klen == 1 && tok[0].first[0] == 'f') {
            if (tok.size() < 4) return kIngestUnsupported;   // < 3 indices: IndexError
            std::vector<int64_t> raw, idx;
            for (size_t t = 1; t < tok.size(); ++t) {
                int64_t v;
                if (!py_int(tok[t].first, tok[t].second, &v)) return kIngestUnsupported;
                const int64_t r = v < 0 ? n_vert + v : v - 1;   // Obj.faces holds this
                const int64_t k = r < 0 ? r + n_vert : r;       // Python negative indexing
                if (k < 0 || k >= n_vert) return kIngestUnsupported;   // IndexError
                raw.push_back(r);
                idx.push_back(k);
            }
            for (size_t j = 1; j + 1 < idx.size(); ++j) {   // fan (a triangle when 3)
                const size_t q3[3] = {0, j, j + 1};
                double n[3], area;
                const double* V = M->vert.data();
                tri_normal_area(V + 3 * idx[0], V + 3 * idx[j], V + 3 * idx[j + 1], n, &area);
                if (!(area != 0.0)) return kIngestDivZero;   // 1/0: ZeroDivisionError
                for (int q = 0; q < 3; ++q) {
                    M->face.push_back(raw[q3[q]]);
                    for (int c = 0; c < 3; ++c) M->tri_v.push_back(V[3 * idx[q3[q]] + c]);
                    M->tri_n.push_back(n[q]);
                }
                M->tri_area.push_back(area);
            }
        } else {
            M->skip_off.push_back((int64_t)line_b);
            M->skip_len.push_back((int64_t)(line_e - line_b));
        }
    }
    return kIngestOk;
}

inline int parse_obj_file(const char* path, MeshOut* M) {
    FILE* f = fopen(path, "rb");
    if (!f) return kIngestIo;
    std::string buf;
    char chunk[1 << 16];
    size_t got;
    while ((got = fread(chunk, 1, sizeof(chunk), f)) > 0) buf.append(chunk, got);
    const bool err = ferror(f) != 0;
    fclose(f);
    if (err) return kIngestIo;
    for (unsigned char c : buf)
        if (c >= 0x80 || c == 0) return kIngestUnsupported;   // non-ASCII: leave to Python's decoder
    return parse_obj_text(buf.data(), buf.size(), M);
}

}  // namespace pt
