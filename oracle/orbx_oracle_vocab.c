/* orbx_oracle_vocab.c -- TEST INFRASTRUCTURE ONLY (see orbx_oracle_vocab.h). */
#define _POSIX_C_SOURCE 200809L
#include "orbx_oracle_vocab.h"

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* FORB::distance, FORB.cpp:81-101 (SWAR popcount over 8 x int32) */
static int forb_distance(const uint8_t* a, const uint8_t* b) {
    int dist = 0;
    for (int i = 0; i < 8; i++) {
        uint32_t x, y;
        memcpy(&x, a + 4 * i, 4);
        memcpy(&y, b + 4 * i, 4);
        uint32_t v = x ^ y;
        v = v - ((v >> 1) & 0x55555555u);
        v = (v & 0x33333333u) + ((v >> 2) & 0x33333333u);
        dist += (int)((((v + (v >> 4)) & 0xF0F0F0Fu) * 0x1010101u) >> 24);
    }
    return dist;
}

void ora_vocab_free(ora_vocab* v) {
    free(v->desc);
    free(v->parent);
    free(v->child_off);
    free(v->child);
    free(v->word_id);
    free(v->weight);
    memset(v, 0, sizeof(*v));
}

/* TemplatedVocabulary::loadFromTextFile, TemplatedVocabulary.h:1338-1424: header
 * "k L scoring weighting", then one node per line "parent isLeaf d0 .. d31 weight"
 * (FORB::fromString reads the 32 bytes as integers, FORB.cpp:120-135); node 0 is the
 * root; a node's children are in file order; leaves get word ids in file order. */
int ora_vocab_load_text(ora_vocab* v, const char* text, size_t len) {
    memset(v, 0, sizeof(*v));
    char* buf = (char*)malloc(len + 1);
    memcpy(buf, text, len);
    buf[len] = 0;
    char* save = NULL;
    char* line = strtok_r(buf, "\n", &save);
    if (!line || sscanf(line, "%d %d %d %d", &v->k, &v->L, &v->scoring, &v->weighting) != 4 || v->k < 0 ||
        v->k > 20 || v->L < 1 || v->L > 10 || v->scoring < 0 || v->scoring > 5 || v->weighting < 0 ||
        v->weighting > 3) {
        free(buf);
        return -1;
    }
    int cap = 1024, n = 1;
    v->desc = (uint8_t*)calloc((size_t)cap, 32);
    v->parent = (int*)calloc((size_t)cap, sizeof(int));
    v->word_id = (int*)malloc(sizeof(int) * (size_t)cap);
    v->weight = (double*)calloc((size_t)cap, sizeof(double));
    v->word_id[0] = 0;
    int nwords = 0;
    while ((line = strtok_r(NULL, "\n", &save)) != NULL) {
        char* p = line;
        while (*p == ' ' || *p == '\t' || *p == '\r') p++;
        if (!*p) continue;  /* empty line (see header) */
        if (n == cap) {
            cap *= 2;
            v->desc = (uint8_t*)realloc(v->desc, (size_t)cap * 32);
            v->parent = (int*)realloc(v->parent, sizeof(int) * (size_t)cap);
            v->word_id = (int*)realloc(v->word_id, sizeof(int) * (size_t)cap);
            v->weight = (double*)realloc(v->weight, sizeof(double) * (size_t)cap);
        }
        char* end;
        const long pid = strtol(p, &end, 10);
        p = end;
        const long leaf = strtol(p, &end, 10);
        p = end;
        for (int i = 0; i < 32; i++) {
            const long b = strtol(p, &end, 10);
            p = end;
            v->desc[(size_t)n * 32 + i] = (uint8_t)b;
        }
        v->weight[n] = strtod(p, &end);
        if (pid < 0 || pid >= n) {
            free(buf);
            ora_vocab_free(v);
            return -1;
        }
        v->parent[n] = (int)pid;
        v->word_id[n] = leaf > 0 ? nwords++ : 0;  /* Node() default word_id 0 */
        n++;
    }
    free(buf);
    v->nnodes = n;
    v->nwords = nwords;
    /* children CSR in file order */
    v->child_off = (int*)calloc((size_t)n + 1, sizeof(int));
    v->child = (int*)malloc(sizeof(int) * (size_t)(n > 1 ? n - 1 : 1));
    for (int i = 1; i < n; i++) v->child_off[v->parent[i] + 1]++;
    for (int i = 0; i < n; i++) v->child_off[i + 1] += v->child_off[i];
    int* fill = (int*)calloc((size_t)n, sizeof(int));
    for (int i = 1; i < n; i++) {
        const int p = v->parent[i];
        v->child[v->child_off[p] + fill[p]++] = i;
    }
    free(fill);
    return 0;
}

/* TemplatedVocabulary::transform(feature, word_id, weight, nid, levelsup),
 * TemplatedVocabulary.h:1220-1259: descend from the root taking the child with the
 * smallest distance (strict <, first child wins ties) until a leaf; *nid = the node
 * reached at level L - levelsup (root if that level is <= 0).  A leaf above that level
 * leaves *nid at the deepest node reached (the reference leaves it uninitialised). */
static void transform_one(const ora_vocab* v, const uint8_t* f, int levelsup, int* word, double* weight, int* nid) {
    const int nid_level = v->L - levelsup;
    int final_id = 0, level = 0;
    *nid = 0;
    do {
        ++level;
        const int c0 = v->child_off[final_id], c1 = v->child_off[final_id + 1];
        int best = v->child[c0];
        double best_d = forb_distance(f, v->desc + (size_t)best * 32);
        for (int c = c0 + 1; c < c1; c++) {
            const int id = v->child[c];
            const double d = forb_distance(f, v->desc + (size_t)id * 32);
            if (d < best_d) {
                best_d = d;
                best = id;
            }
        }
        final_id = best;
        if (level <= nid_level) *nid = final_id;
    } while (v->child_off[final_id] != v->child_off[final_id + 1]);
    if (nid_level <= 0) *nid = 0;
    *word = v->word_id[final_id];
    *weight = v->weight[final_id];
}

int ora_vocab_transform_features(const ora_vocab* v, const uint8_t* desc, int n, int levelsup, int32_t* word,
                                 double* weight, int32_t* node) {
    for (int i = 0; i < n; i++) {
        int w, nid;
        double wt;
        transform_one(v, desc + (size_t)i * 32, levelsup, &w, &wt, &nid);
        word[i] = w;
        weight[i] = wt;
        node[i] = nid;
    }
    return 0;
}

typedef struct {
    int key;  /* word or node id */
    int idx;  /* feature index */
    double w;
} kv;

static int kv_cmp(const void* a, const void* b) {
    const kv* x = (const kv*)a;
    const kv* y = (const kv*)b;
    if (x->key != y->key) return x->key < y->key ? -1 : 1;
    return x->idx < y->idx ? -1 : (x->idx > y->idx);
}

/* transform(features, BowVector&, FeatureVector&, levelsup), TemplatedVocabulary.h:
 * 1127-1186 + BowVector::addWeight / addIfNotExist / normalize (BowVector.cpp) +
 * FeatureVector::addFeature (FeatureVector.cpp:31-45). */
int ora_vocab_transform(const ora_vocab* v, const uint8_t* desc, int n, int levelsup, int32_t* bow_word,
                        double* bow_value, int* nbow, int32_t* fv_node, int32_t* fv_off, int32_t* fv_idx, int* nfv) {
    *nbow = 0;
    *nfv = 0;
    if (v->nwords == 0 || n <= 0) {  /* empty(): no words */
        fv_off[0] = 0;
        return 0;
    }
    kv* words = (kv*)malloc(sizeof(kv) * (size_t)n);
    kv* nodes = (kv*)malloc(sizeof(kv) * (size_t)n);
    int nw = 0;
    for (int i = 0; i < n; i++) {
        int w, nid;
        double wt;
        transform_one(v, desc + (size_t)i * 32, levelsup, &w, &wt, &nid);
        if (wt > 0) {  /* not stopped */
            words[nw].key = w;
            words[nw].idx = i;
            words[nw].w = wt;
            nodes[nw].key = nid;
            nodes[nw].idx = i;
            nodes[nw].w = 0;
            nw++;
        }
    }
    qsort(words, (size_t)nw, sizeof(kv), kv_cmp);
    qsort(nodes, (size_t)nw, sizeof(kv), kv_cmp);
    /* BowVector: TF / TF_IDF (0, 1) accumulate in feature order, IDF / BINARY (2, 3)
     * keep the first */
    const int accumulate = v->weighting == 0 || v->weighting == 1;
    int nb = 0;
    for (int j = 0; j < nw; j++) {
        if (nb > 0 && bow_word[nb - 1] == words[j].key) {
            if (accumulate) bow_value[nb - 1] += words[j].w;
        } else {
            bow_word[nb] = words[j].key;
            bow_value[nb] = words[j].w;
            nb++;
        }
    }
    /* normalisation: scoring L1/ChiSquare/KL/Bhattacharyya -> L1, L2 -> L2, DotProduct
     * -> none (ScoringObject.h:74-89); TF / TF_IDF without normalisation divide by
     * the word count (TemplatedVocabulary.h:1162-1168) */
    const int must = v->scoring != 5;
    if (must) {
        double norm = 0.0;
        if (v->scoring == 1) {
            /* fused, as the reference builds it: g++ contracts C++ even under -std=c++11
             * (contraction is off by default only for ISO C), and BowVector.cpp compiled
             * with DBoW2's -O3 -march=native holds one vfmadd, in this loop
             * (tests/test_vocab_ref.py runs that build) */
            for (int j = 0; j < nb; j++) norm = fma(bow_value[j], bow_value[j], norm);
            norm = sqrt(norm);
        } else {
            for (int j = 0; j < nb; j++) norm += fabs(bow_value[j]);
        }
        if (norm > 0.0)
            for (int j = 0; j < nb; j++) bow_value[j] /= norm;
    } else if (accumulate && nb > 0) {
        const double nd = nb;
        for (int j = 0; j < nb; j++) bow_value[j] /= nd;
    }
    *nbow = nb;
    /* FeatureVector */
    int nf = 0;
    for (int j = 0; j < nw; j++) {
        if (nf == 0 || fv_node[nf - 1] != nodes[j].key) {
            fv_node[nf] = nodes[j].key;
            fv_off[nf] = j;
            nf++;
        }
        fv_idx[j] = nodes[j].idx;
    }
    fv_off[nf] = nw;
    *nfv = nf;
    free(words);
    free(nodes);
    return 0;
}
