/*
 * TEST INFRASTRUCTURE ONLY (see oracle.h).  CPU restatement of the Quickstart chip join:
 *
 *   trips.join(chips, grid_pointascellid(point, res) == chip.index_id)
 *        .where(chip.is_core || st_contains(chip.wkb, point))
 *
 * (reference notebooks/examples/python/QuickstartNotebook.py:205-219;
 *  sql/join/PointInPolygonJoin.scala:68-84).  Each matching (point, chip) pair is one output
 * row; counts[] accumulates rows per chip polygon key (the groupBy(zone).count() of BASELINE.md).
 * Cell ids: H3 via h3.c (H3IndexSystem.pointToIndex), BNG via bng.c (BNGIndexSystem.pointToIndex).
 * Chip WKBs are decoded once up front (the reference re-decodes per pair; same answers).
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

typedef struct {
    const oracle_chips* chips;
    void** parsed; /* decoded chip WKBs (NULL: undecodable -> contains false) */
    int64_t* order; /* chip indices sorted by (index_id, original position) */
    int grid, res, jdk;
    const double* x;
    const double* y;
    int64_t lo, hi;
    int64_t* counts;
    int64_t n_polygons;
    int64_t* pair_row;
    int32_t* pair_key;
    int64_t cap, n_pairs;
} job;

static const oracle_chips* g_sort_chips;
static int cmp_chip(const void* a, const void* b) {
    int64_t ia = *(const int64_t*)a, ib = *(const int64_t*)b;
    int64_t ka = g_sort_chips->index_id[ia], kb = g_sort_chips->index_id[ib];
    if (ka != kb) return ka < kb ? -1 : 1;
    return ia < ib ? -1 : (ia > ib);
}

static int64_t lower_bound(const oracle_chips* c, const int64_t* order, int64_t n, int64_t key) {
    int64_t lo = 0, hi = n;
    while (lo < hi) {
        int64_t mid = (lo + hi) / 2;
        if (c->index_id[order[mid]] < key)
            lo = mid + 1;
        else
            hi = mid;
    }
    return lo;
}

static void* run_job(void* arg) {
    job* j = (job*)arg;
    const oracle_chips* c = j->chips;
    for (int64_t i = j->lo; i < j->hi; i++) {
        int64_t cell;
        if (j->grid == 0) {
            cell = oracle_h3_geo_to_h3(oracle_to_radians(j->y[i], j->jdk), oracle_to_radians(j->x[i], j->jdk),
                                       j->res);
        } else {
            int err;
            cell = oracle_bng_point_to_index(j->x[i], j->y[i], j->res, &err);
            if (err) continue; /* NaN row: the reference raises; the join drops it here */
        }
        int64_t k = lower_bound(c, j->order, c->n_chips, cell);
        for (; k < c->n_chips && c->index_id[j->order[k]] == cell; k++) {
            int64_t ci = j->order[k];
            int hit = c->is_core[ci];
            if (!hit) {
                hit = j->parsed[ci] && oracle_parsed_contains(j->parsed[ci], j->x[i], j->y[i]) == 1;
            }
            if (hit) {
                int32_t key = c->polygon_key[ci];
                if (key >= 0 && key < j->n_polygons) j->counts[key]++;
                if (j->pair_row && j->n_pairs < j->cap) {
                    j->pair_row[j->n_pairs] = i;
                    j->pair_key[j->n_pairs] = key;
                }
                j->n_pairs++;
            }
        }
    }
    return NULL;
}

/* Brute-force st_contains join (the reference's expected count in MosaicFrameBehaviors.scala:157-162):
 * counts[polygon_key[g]] += #points p with contains(geometry g, p), every geometry tested. */
int64_t oracle_brute_force_count(const oracle_chips* geoms, const double* x, const double* y, int64_t n,
                                 int64_t* counts, int64_t n_polygons) {
    int64_t total = 0;
    for (int64_t g = 0; g < geoms->n_chips; g++) {
        void* pg = oracle_wkb_parse(geoms->wkb + geoms->wkb_offsets[g], geoms->wkb_offsets[g + 1] - geoms->wkb_offsets[g]);
        if (!pg) continue;
        int32_t key = geoms->polygon_key[g];
        for (int64_t i = 0; i < n; i++) {
            if (oracle_parsed_contains(pg, x[i], y[i]) == 1) {
                if (key >= 0 && key < n_polygons) counts[key]++;
                total++;
            }
        }
        oracle_parsed_free(pg);
    }
    return total;
}

int64_t oracle_pip_join(const oracle_chips* chips, int grid, int res, int jdk, const double* x,
                        const double* y, int64_t n, int64_t* counts, int64_t n_polygons,
                        int64_t* pair_row, int32_t* pair_key, int64_t cap, int n_threads) {
    int64_t* order = malloc(sizeof(int64_t) * (chips->n_chips ? chips->n_chips : 1));
    for (int64_t i = 0; i < chips->n_chips; i++) order[i] = i;
    g_sort_chips = chips;
    qsort(order, chips->n_chips, sizeof(int64_t), cmp_chip);
    void** parsed = calloc(chips->n_chips ? chips->n_chips : 1, sizeof(void*));
    for (int64_t i = 0; i < chips->n_chips; i++)
        if (!chips->is_core[i])
            parsed[i] = oracle_wkb_parse(chips->wkb + chips->wkb_offsets[i],
                                         chips->wkb_offsets[i + 1] - chips->wkb_offsets[i]);
    if (n_threads < 1) n_threads = 1;
    if (pair_row) n_threads = 1; /* pairs are emitted in row order by one thread */
    job* jobs = calloc(n_threads, sizeof(job));
    pthread_t* th = calloc(n_threads, sizeof(pthread_t));
    int64_t total = 0;
    for (int t = 0; t < n_threads; t++) {
        job* j = &jobs[t];
        j->chips = chips;
        j->parsed = parsed;
        j->order = order;
        j->grid = grid;
        j->res = res;
        j->jdk = jdk;
        j->x = x;
        j->y = y;
        j->lo = n * t / n_threads;
        j->hi = n * (t + 1) / n_threads;
        j->counts = calloc(n_polygons > 0 ? n_polygons : 1, sizeof(int64_t));
        j->n_polygons = n_polygons;
        j->pair_row = pair_row;
        j->pair_key = pair_key;
        j->cap = cap;
        if (n_threads == 1)
            run_job(j);
        else
            pthread_create(&th[t], NULL, run_job, j);
    }
    for (int t = 0; t < n_threads; t++) {
        if (n_threads > 1) pthread_join(th[t], NULL);
        for (int64_t p = 0; p < n_polygons; p++) counts[p] += jobs[t].counts[p];
        total += jobs[t].n_pairs;
        free(jobs[t].counts);
    }
    free(jobs);
    free(th);
    for (int64_t i = 0; i < chips->n_chips; i++) oracle_parsed_free(parsed[i]);
    free(parsed);
    free(order);
    return total;
}
