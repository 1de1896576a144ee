// sanitize_main.cpp — TEST INFRASTRUCTURE.  An ASan + UBSan executable
// (tests/hostcheck/Makefile target `sanitize`) over the host code that ships
// inside libpt_hip.so and handles untrusted input or builds trees:
//   * pt_ingest.h  — the native OBJ reader (scene_reader.py:49-104), on the
//     Cornell meshes, random valid meshes and mutated / truncated texts;
//   * pt_prepare.h — scene preparation: plane units, the binned-SAH BVH, its
//     4-wide quantised form (QNode), the 64-B leaf records — on Cornell plus
//     random meshes of several sizes;
//   * the kernel's per-lane code (pt_path.h, pt_wavefront.h) through the
//     host-build entry points of pt_hostcheck.cpp: single-kernel and
//     wavefront renders, the BVH reachability check and the filter self-test.
// Exit 0 = no sanitizer report (the sanitizers abort on the first one) and
// every consistency check passed.  Usage: sanitize <scenes/cornell dir>
#include "pt_hostcheck.cpp"
#include "../../pathtracerpython_amd/csrc/pt_ingest.h"

#include <cmath>
#include <cstdio>
#include <string>
#include <vector>

// the C oracle (oracle/pt_oracle.c), built with the same sanitizers
extern "C" int oracle_render(const pt_scene_desc* d, const pt_render_params* p, const int64_t* pixels,
                             int64_t n_pixels, int n_threads, double* out, pt_stats* stats);

namespace {

struct Obj {
    std::vector<double> tri_v, tri_n, tri_area;
};

bool load(const std::string& path, Obj* o) {
    MeshOut M;
    if (parse_obj_file(path.c_str(), &M) != kIngestOk) return false;
    o->tri_v = M.tri_v;
    o->tri_n = M.tri_n;
    o->tri_area = M.tri_area;
    return true;
}

// random valid mesh as OBJ text (small triangles inside the Cornell box)
std::string random_obj(int n, uint64_t seed, double sigma) {
    std::mt19937_64 rng(seed);
    std::uniform_real_distribution<double> ux(-3.5, 3.5), uz(-31.0, -18.0);
    std::normal_distribution<double> N(0.0, sigma);
    std::string s = "# random mesh\n";
    char buf[128];
    for (int i = 0; i < n; ++i) {
        const double c[3] = {ux(rng), ux(rng), uz(rng)};
        for (int v = 0; v < 3; ++v) {
            snprintf(buf, sizeof buf, "v %.17g %.17g %.17g\n", c[0] + N(rng), c[1] + N(rng), c[2] + N(rng));
            s += buf;
        }
    }
    for (int i = 0; i < n; ++i) {
        snprintf(buf, sizeof buf, "f %d %d %d\n", 3 * i + 1, 3 * i + 2, 3 * i + 3);
        s += buf;
    }
    return s;
}

int fuzz_ingest(const std::string& base, uint64_t seed) {
    // every prefix of a small valid text, then random byte mutations and
    // token splices of a larger one: the reader may refuse, never misbehave
    std::mt19937_64 rng(seed);
    int ok = 0;
    const std::string small = "v 0 0 0\nv 1 0 0\r\nv 0 1 0\n# c\nf 1 2 3\nf -1 -2 -3 # x\n\tvt 1 2\n";
    for (size_t n = 0; n <= small.size(); ++n) {
        MeshOut M;
        ok += parse_obj_text(small.data(), n, &M) == kIngestOk;
    }
    static const char* splice[] = {"f", "v", " ", "\t", "\n", "\r", "#", "-", "+", ".", "e", "1e308",
                                   "-0", "nan", "inf", "9999999999999999999", "0x1p3", "1_0", "/", "f 1 1 1"};
    for (int it = 0; it < 3000; ++it) {
        std::string t = base;
        const int edits = 1 + (int)(rng() % 8);
        for (int e = 0; e < edits && !t.empty(); ++e) {
            const size_t pos = rng() % t.size();
            switch (rng() % 4) {
                case 0: t[pos] = (char)(32 + rng() % 95); break;
                case 1: t.erase(pos, 1 + rng() % 16); break;
                case 2: t.insert(pos, splice[rng() % (sizeof splice / sizeof *splice)]); break;
                default: t.resize(pos); break;
            }
        }
        MeshOut M;
        ok += parse_obj_text(t.data(), t.size(), &M) == kIngestOk;
    }
    return ok;
}

struct SceneBuild {
    std::vector<double> tri_v, tri_n, tri_area, mat;
    std::vector<int32_t> tri_obj;
    pt_scene_desc d{};
    int n_obj = 0;
    void add(const Obj& o, int obj) {
        tri_v.insert(tri_v.end(), o.tri_v.begin(), o.tri_v.end());
        tri_n.insert(tri_n.end(), o.tri_n.begin(), o.tri_n.end());
        tri_area.insert(tri_area.end(), o.tri_area.begin(), o.tri_area.end());
        for (size_t i = 0; i < o.tri_area.size(); ++i) tri_obj.push_back(obj);
    }
    void finish(int n_obj_tri) {
        d.n_tri = (int32_t)tri_area.size();
        d.n_obj_tri = n_obj_tri;
        d.n_obj = n_obj;
        d.tri_v = tri_v.data();
        d.tri_n = tri_n.data();
        d.tri_area = tri_area.data();
        d.tri_obj = tri_obj.data();
        d.mat = mat.data();
        d.eye[0] = 0; d.eye[1] = 0; d.eye[2] = 5.7;
        d.ortho[0] = -1; d.ortho[1] = -1; d.ortho[2] = 1; d.ortho[3] = 1;
        d.ambient = 0.5;
        d.light_rgb[0] = d.light_rgb[1] = d.light_rgb[2] = 1.0;
    }
};

#define CHECK(c)                                                        \
    do {                                                                \
        if (!(c)) {                                                     \
            fprintf(stderr, "sanitize: check failed: %s (line %d)\n", #c, __LINE__); \
            return 1;                                                   \
        }                                                               \
    } while (0)

}  // namespace

int main(int argc, char** argv) {
    if (argc < 2) {
        fprintf(stderr, "usage: sanitize <scenes/cornell dir>\n");
        return 2;
    }
    const std::string dir = argv[1];
    const char* walls[] = {"leftwall.obj", "rightwall.obj", "floor.obj", "back.obj", "ceiling.obj",
                           "cube1.obj", "cube2.obj"};
    const double mats[7][8] = {{1, 0, 0, .3, .7, 0, 0, 5}, {0, 1, 0, .3, .7, 0, 0, 5},
                               {1, 1, 1, .3, .7, 0, 0, 5}, {1, 1, 1, .3, .7, 0, 0, 5},
                               {1, 1, 1, .3, .7, 0, 0, 5}, {1, 1, 1, .3, .7, .9, 0, 5},
                               {1, 1, 1, .3, .7, .6, 0, 5}};
    std::vector<Obj> objs(7);
    for (int i = 0; i < 7; ++i) CHECK(load(dir + "/" + walls[i], &objs[i]));
    Obj light;
    CHECK(load(dir + "/luzcornell.obj", &light));
    CHECK(!load(dir + "/does-not-exist.obj", &light) || true);

    // 1. ingest fuzz (random mesh text as the mutation base)
    const int fz = fuzz_ingest(random_obj(40, 7, 0.3), 11);
    printf("ingest fuzz: %d texts accepted\n", fz);

    // 2. scenes: Cornell, and Cornell + random meshes (BVH) of several sizes
    const int sizes[] = {0, 70, 300, 2000};
    for (int si = 0; si < 4; ++si) {
        SceneBuild S;
        int obj = 0;
        for (int i = 0; i < 7; ++i) {
            S.add(objs[i], obj++);
            S.mat.insert(S.mat.end(), mats[i], mats[i] + 8);
        }
        Obj rnd;
        if (sizes[si]) {
            const std::string t = random_obj(sizes[si], 100 + si, si == 3 ? 0.05 : 0.5);
            MeshOut M;
            CHECK(parse_obj_text(t.data(), t.size(), &M) == kIngestOk);
            rnd.tri_v = M.tri_v; rnd.tri_n = M.tri_n; rnd.tri_area = M.tri_area;
            S.add(rnd, obj++);
            const double m[8] = {.2, .5, .9, .3, .6, .4, 0, 3};
            S.mat.insert(S.mat.end(), m, m + 8);
        }
        S.n_obj = obj;
        const int n_obj_tri = (int)S.tri_area.size();
        S.add(light, obj);
        S.finish(n_obj_tri);

        int32_t info[6] = {0, 0, 0, 0, 0, 0};
        CHECK(hc_bvh_info(&S.d, info) == 0);
        int64_t fs[8] = {0};
        CHECK(hc_filter_selftest(&S.d, 20000, 5 + si, fs) == 0);
        CHECK(fs[0] == 0 && fs[4] == 0);   // no wrong certain verdict
        if (sizes[si]) {
            int64_t bc[4] = {0};
            CHECK(hc_bvh_check(&S.d, 4000, 9 + si, bc) == 0);
            CHECK(bc[0] == 0 && bc[1] == 0);
        }
        pt_render_params p{};
        p.width = 12; p.height = 10; p.spp = 2; p.bounces = 4; p.seed = 3 + si;
        p.flags = si == 2 ? PT_FLAG_RR : 0; p.rr_depth = 2;
        p.row_begin = 0; p.row_end = p.height; p.row_step = 1; p.row_phase = 0;
        std::vector<double> a(p.width * p.height * 3), b(a.size()), c(a.size());
        uint64_t cnt[8];
        CHECK(hc_render(&S.d, &p, 0, a.data(), cnt) == 0);
        CHECK(hc_render(&S.d, &p, 1, b.data(), nullptr) == 0);
        CHECK(a == b);   // hybrid == forced f64, bit for bit
        {   // the oracle (2 threads) on every pixel, to rounding
            std::vector<int64_t> pix;
            for (int ix = 0; ix < p.width; ++ix)
                for (int iy = 0; iy < p.height; ++iy) pix.push_back((int64_t)ix * p.height + iy);
            std::vector<double> o(pix.size() * 3);
            pt_stats ost;
            CHECK(oracle_render(&S.d, &p, pix.data(), (int64_t)pix.size(), 2, o.data(), &ost) == 0);
            double err = 0.0;
            for (size_t i = 0; i < pix.size(); ++i) {
                const int ix = (int)(pix[i] / p.height), iy = (int)(pix[i] % p.height);
                for (int c = 0; c < 3; ++c)
                    err = std::max(err, std::fabs(o[3 * i + c] - a[((size_t)(p.height - 1 - iy) * p.width + ix) * 3 + c]));
            }
            CHECK(err <= 1e-12);
        }
        if (sizes[si]) {
            int32_t steps = 0;
            int64_t ws[8];
            CHECK(hc_render_wavefront(&S.d, &p, c.data(), &steps, ws) == 0);
            CHECK(a == c);   // wavefront == single kernel
        }
        printf("scene %d: %d tris, bnodes %d depth %d qnodes %d, %llu tests\n", si, S.d.n_tri,
               info[0], info[1], info[2], (unsigned long long)(cnt[0] + cnt[1]));
    }
    printf("sanitize: OK\n");
    return 0;
}
