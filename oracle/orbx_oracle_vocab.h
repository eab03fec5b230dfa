/* orbx_oracle_vocab.h -- TEST INFRASTRUCTURE ONLY: CPU restatement of DBoW2's
 * TemplatedVocabulary<FORB::TDescriptor, FORB> text loading and transform
 * (Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h:1127-1259, 1338-1424; BowVector.cpp;
 * FeatureVector.cpp:31-45; FORB.cpp:81-135).  Parity status: "parity unpinned" (the
 * reference cannot be built here and ships no vocabulary or tests). */
#ifndef ORBX_ORACLE_VOCAB_H
#define ORBX_ORACLE_VOCAB_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
    int k, L, scoring, weighting;  /* header line: k L scoring weighting */
    int nnodes, nwords;
    uint8_t* desc;                 /* nnodes x 32 */
    int* parent;
    int* child_off;                /* CSR: children of node i at child[child_off[i] .. child_off[i+1]) */
    int* child;
    int* word_id;                  /* 0 for nodes not flagged as leaves (Node() default) */
    double* weight;
} ora_vocab;

/* loadFromTextFile on an in-memory text.  Lines that are empty (the trailing newline)
 * are skipped (the reference would add a node with uninitialised contents, see
 * DESIGN.md).  Returns 0 on success. */
int ora_vocab_load_text(ora_vocab* v, const char* text, size_t len);
void ora_vocab_free(ora_vocab* v);

/* transform(features, BowVector, FeatureVector, levelsup) for one frame.  BowVector as
 * (bow_word[j], bow_value[j]) ascending by word; FeatureVector as CSR (fv_node[j]
 * ascending, features fv_idx[fv_off[j] .. fv_off[j+1]) ascending).  Capacities n.
 * Returns 0. */
int ora_vocab_transform(const ora_vocab* v, const uint8_t* desc, int n, int levelsup, int32_t* bow_word,
                        double* bow_value, int* nbow, int32_t* fv_node, int32_t* fv_off, int32_t* fv_idx, int* nfv);

/* transform(feature, word_id, weight, nid, levelsup) for each of n descriptors
 * (TemplatedVocabulary.h:1220-1259): the per-feature tree walk the frame transform
 * aggregates.  Returns 0. */
int ora_vocab_transform_features(const ora_vocab* v, const uint8_t* desc, int n, int levelsup, int32_t* word,
                                 double* weight, int32_t* node);

#ifdef __cplusplus
}
#endif
#endif
