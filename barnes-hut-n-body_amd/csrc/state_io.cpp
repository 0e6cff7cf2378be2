// On-disk state format (SURVEY §5 "Checkpoint / resume", §8f row 3): the caller-visible state
// of a PhysicsEngine -- its Config fields and its body list (BHA:21-25, 287-349) -- as one
// little-endian file, so a run can stop and resume bit for bit.  Layout (all little-endian):
//
//   offset  size        field
//   0       8           magic "BHSTATE1"
//   8       4           uint32 size of the block from byte 16 to the body arrays (= 64): the
//                       body arrays start at byte 16 + this field = 80
//   12      4           uint32 flags (0)
//   16      8 x 4       double G, dt, theta, soft2                (CFG:11,14,23,20)
//   48      4 x 2       int32 width_px, height_px                 (CFG:5,8)
//   56      8 x 2       double merge_max_mass, merge_min_dist     (BHA:315,321)
//   72      8           int64 N
//   80      8 N x 5     double x[N], y[N], vx[N], vy[N], m[N]     (the caller's list order)
//
// The engine's internal Morton order is not part of the state: the tree is a function of the
// point set and the list order (BHA:363), so loading = bh_set_params + bh_reset_bodies of the
// saved list reproduces every later step exactly.
#include <cstdio>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "bh_engine.h"

namespace bh {
void set_error(bh_engine *e, const std::string &msg);  // engine.cpp
}

namespace {

constexpr char kMagic[8] = {'B', 'H', 'S', 'T', 'A', 'T', 'E', '1'};
constexpr uint32_t kHeaderBytes = 64;

static_assert(sizeof(double) == 8 && sizeof(int64_t) == 8, "fp64 / int64 state words");

bool little_endian() {
    const uint16_t one = 1;
    uint8_t b;
    std::memcpy(&b, &one, 1);
    return b == 1;
}

struct File {
    std::FILE *f = nullptr;
    ~File() {
        if (f) std::fclose(f);
    }
};

}  // namespace

extern "C" {

int bh_save_state(bh_engine *e, const char *path) {
    if (!e || !path) return BH_E_INVALID;
    if (!little_endian()) return BH_E_STATE;
    bh_params p;
    int rc = bh_get_params(e, &p);
    if (rc != BH_OK) return rc;
    const int64_t n = bh_num_bodies(e);
    std::vector<double> a((size_t)(5 * n) + 1);
    int64_t got = 0;
    rc = bh_get_bodies(e, a.data(), a.data() + n, a.data() + 2 * n, a.data() + 3 * n,
                       a.data() + 4 * n, n, &got);
    if (rc != BH_OK) return rc;
    File out;
    const std::string tmp = std::string(path) + ".tmp";
    out.f = std::fopen(tmp.c_str(), "wb");
    if (!out.f) {
        bh::set_error(e, "bh_save_state: cannot create " + tmp);
        return BH_E_INVALID;
    }
    uint8_t hdr[80] = {};
    std::memcpy(hdr, kMagic, 8);
    std::memcpy(hdr + 8, &kHeaderBytes, 4);
    std::memcpy(hdr + 16, &p.G, 8);
    std::memcpy(hdr + 24, &p.dt, 8);
    std::memcpy(hdr + 32, &p.theta, 8);
    std::memcpy(hdr + 40, &p.soft2, 8);
    std::memcpy(hdr + 48, &p.width_px, 4);
    std::memcpy(hdr + 52, &p.height_px, 4);
    std::memcpy(hdr + 56, &p.merge_max_mass, 8);
    std::memcpy(hdr + 64, &p.merge_min_dist, 8);
    std::memcpy(hdr + 72, &n, 8);
    bool ok = std::fwrite(hdr, 1, sizeof(hdr), out.f) == sizeof(hdr) &&
              (n == 0 || std::fwrite(a.data(), sizeof(double), (size_t)(5 * n), out.f) ==
                             (size_t)(5 * n));
    ok = std::fclose(out.f) == 0 && ok;
    out.f = nullptr;
    if (!ok || std::rename(tmp.c_str(), path) != 0) {
        std::remove(tmp.c_str());
        bh::set_error(e, std::string("bh_save_state: cannot write ") + path);
        return BH_E_INVALID;
    }
    return BH_OK;
}

int bh_load_state(bh_engine *e, const char *path) {
    if (!e || !path) return BH_E_INVALID;
    if (!little_endian()) return BH_E_STATE;
    File in;
    in.f = std::fopen(path, "rb");
    auto bad = [&](const char *why) {
        bh::set_error(e, std::string("bh_load_state: ") + path + ": " + why);
        return BH_E_INVALID;
    };
    if (!in.f) return bad("cannot open");
    uint8_t hdr[80];
    if (std::fread(hdr, 1, sizeof(hdr), in.f) != sizeof(hdr) || std::memcmp(hdr, kMagic, 8) != 0)
        return bad("not a BHSTATE1 file");
    uint32_t hb = 0;
    std::memcpy(&hb, hdr + 8, 4);
    if (hb != kHeaderBytes) return bad("unknown header block size");
    bh_params p;
    std::memcpy(&p.G, hdr + 16, 8);
    std::memcpy(&p.dt, hdr + 24, 8);
    std::memcpy(&p.theta, hdr + 32, 8);
    std::memcpy(&p.soft2, hdr + 40, 8);
    std::memcpy(&p.width_px, hdr + 48, 4);
    std::memcpy(&p.height_px, hdr + 52, 4);
    std::memcpy(&p.merge_max_mass, hdr + 56, 8);
    std::memcpy(&p.merge_min_dist, hdr + 64, 8);
    int64_t n = 0;
    std::memcpy(&n, hdr + 72, 8);
    if (n < 0 || n > ((int64_t)1 << 40)) return bad("body count out of range");
    // the file must be exactly the header plus 5 N doubles -- checked before allocating, so a
    // corrupt or hostile N cannot ask for memory the file does not back
    if (std::fseek(in.f, 0, SEEK_END) != 0) return bad("cannot seek");
    const long len = std::ftell(in.f);
    if (len < 0 || (int64_t)len != 80 + 40 * n) return bad("file length does not match N");
    if (std::fseek(in.f, 80, SEEK_SET) != 0) return bad("cannot seek");
    std::vector<double> a;
    try {
        a.resize((size_t)(5 * n) + 1);
    } catch (const std::bad_alloc &) {
        return bad("not enough host memory for the body arrays");
    }
    if (n > 0 && std::fread(a.data(), sizeof(double), (size_t)(5 * n), in.f) != (size_t)(5 * n))
        return bad("truncated body arrays");
    int rc = bh_set_params(e, &p);
    if (rc != BH_OK) return rc;
    return bh_reset_bodies(e, n, a.data(), a.data() + n, a.data() + 2 * n, a.data() + 3 * n,
                           a.data() + 4 * n);
}

}  // extern "C"
