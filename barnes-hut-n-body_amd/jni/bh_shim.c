/* The Kotlin drop-in's native logic over the C-ABI (see bh_shim.h). */
#include "bh_shim.h"

#include <stddef.h>
#include <stdlib.h>

/* BH_DEVICES="0,1,2" (repeats allowed) overrides the mask with an explicit device list */
static int create_from_env(const bh_params *p, const char *list, bh_engine **out) {
    int32_t dev[64];
    int32_t n = 0;
    const char *q = list;
    while (*q && n < 64) {
        char *end = NULL;
        const long d = strtol(q, &end, 10);
        if (end == q || d < 0 || d > 1023) return BH_E_INVALID;
        dev[n++] = (int32_t)d;
        q = *end == ',' ? end + 1 : end;
        if (*end && *end != ',') return BH_E_INVALID;
    }
    if (n == 0 || *q) return BH_E_INVALID;
    return bh_create_multi_list(p, dev, n, out);
}

int bh_shim_create(uint32_t device_mask, bh_engine **out) {
    bh_params p;
    bh_default_params(&p); /* Config.kt defaults (CFG:5-23); setParams follows before any step */
    *out = NULL;
    const char *list = getenv("BH_DEVICES");
    int rc = list && *list ? create_from_env(&p, list, out) : bh_create_multi(&p, device_mask, out);
    /* getBodies after every frame (PNL:302); two buffers: the shim compares its list against the
     * mapped one while the next step runs */
    if (rc == BH_OK) rc = bh_set_mirror(*out, 2);
    if (rc != BH_OK && *out) {
        bh_destroy(*out);
        *out = NULL;
    }
    return rc;
}

int bh_shim_set_params(bh_engine *e, double G, double dt, double theta, double soft2,
                       int32_t width_px, int32_t height_px, double merge_max_mass,
                       double merge_min_dist) {
    bh_params p;
    p.G = G;
    p.dt = dt;
    p.theta = theta;
    p.soft2 = soft2;
    p.width_px = width_px;
    p.height_px = height_px;
    p.merge_max_mass = merge_max_mass;
    p.merge_min_dist = merge_min_dist;
    return bh_set_params(e, &p);
}

int bh_shim_reset(bh_engine *e, int64_t n, const double *soa) {
    if (n < 0 || (n > 0 && !soa)) return BH_E_INVALID;
    return bh_reset_bodies(e, n, soa, soa + n, soa + 2 * n, soa + 3 * n, soa + 4 * n);
}

int bh_shim_step(bh_engine *e, int32_t k) { return bh_step(e, k); }

int bh_shim_step_begin(bh_engine *e, int32_t k) { return bh_step_begin(e, k); }

int bh_shim_positions(bh_engine *e, const double *soa[5], int64_t *n, int64_t *n_before,
                      const int32_t **survivors) {
    if (!soa || !n || !n_before || !survivors) return BH_E_INVALID;
    const double *x = NULL, *y = NULL, *m = NULL;
    const uint32_t *sv = NULL;
    const int rc = bh_step_positions(e, &x, &y, &m, &sv, n, n_before);
    if (rc != BH_OK) return rc;
    const ptrdiff_t stride = y - x; /* the planes of one buffer: x, y, vx, vy, m */
    soa[0] = x;
    soa[1] = y;
    soa[2] = x + 2 * stride;
    soa[3] = x + 3 * stride;
    soa[4] = m;
    *survivors = (const int32_t *)sv; /* indices < 2^31: the Kotlin IntBuffer */
    return BH_OK;
}

int bh_shim_survivors(bh_engine *e, const int32_t **survivors, int64_t *n, int64_t *n_before) {
    if (!survivors || !n || !n_before) return BH_E_INVALID;
    const uint32_t *sv = NULL;
    const int rc = bh_step_positions(e, NULL, NULL, NULL, &sv, n, n_before);
    if (rc == BH_OK) *survivors = (const int32_t *)sv;
    return rc;
}

int bh_shim_step_end(bh_engine *e) { return bh_step_end(e); }

int bh_shim_get(bh_engine *e, double *soa, int64_t cap, int64_t *n) {
    const int64_t cnt = bh_num_bodies(e);
    if (n) *n = cnt;
    if (cnt < 0) return BH_E_INVALID;
    if (cap < cnt || (cnt > 0 && !soa)) return BH_E_CAPACITY;
    int64_t got = 0;
    if (cnt == 0) return BH_OK;
    return bh_get_bodies(e, soa, soa + cnt, soa + 2 * cnt, soa + 3 * cnt, soa + 4 * cnt, cnt, &got);
}

int bh_shim_map(bh_engine *e, const double *soa[5], int64_t *n) {
    if (!soa || !n) return BH_E_INVALID;
    return bh_map_bodies(e, &soa[0], &soa[1], &soa[2], &soa[3], &soa[4], n);
}

int bh_shim_quads(bh_engine *e, double *q, int64_t cap, int64_t *nq) {
    int64_t need = 0;
    int rc = bh_get_quads(e, NULL, NULL, NULL, 0, &need);
    if (rc != BH_OK && rc != BH_E_CAPACITY) return rc;
    if (nq) *nq = need;
    if (cap < need || (need > 0 && !q)) return BH_E_CAPACITY;
    if (need == 0) return BH_OK;
    double *tmp = (double *)malloc(sizeof(double) * 3 * (size_t)need);
    if (!tmp) return BH_E_INVALID;
    int64_t got = 0;
    rc = bh_get_quads(e, tmp, tmp + need, tmp + 2 * need, need, &got);
    if (rc == BH_OK) {
        for (int64_t i = 0; i < got; ++i) { /* QuadList reads triples */
            q[3 * i] = tmp[i];
            q[3 * i + 1] = tmp[need + i];
            q[3 * i + 2] = tmp[2 * need + i];
        }
        if (nq) *nq = got;
    }
    free(tmp);
    return rc;
}

int bh_shim_last_removed(const bh_engine *e, int32_t *idx, int64_t cap, int64_t *count) {
    int64_t need = 0;
    int rc = bh_last_removed(e, NULL, 0, &need);
    if (rc != BH_OK && rc != BH_E_CAPACITY) return rc;
    if (count) *count = need;
    if (cap < need || (need > 0 && !idx)) return BH_E_CAPACITY;
    if (need == 0) return BH_OK;
    int64_t *tmp = (int64_t *)malloc(sizeof(int64_t) * (size_t)need);
    if (!tmp) return BH_E_INVALID;
    rc = bh_last_removed(e, tmp, need, &need);
    if (rc == BH_OK)
        for (int64_t i = 0; i < need; ++i) idx[i] = (int32_t)tmp[i]; /* list sizes fit a jint */
    free(tmp);
    return rc;
}
