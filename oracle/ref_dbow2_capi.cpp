// ref_dbow2_capi.cpp -- TEST INFRASTRUCTURE ONLY.  A C entry point over the reference's
// own DBoW2 BowVector / FeatureVector, compiled from the reference sources where they lie
// (Thirdparty/DBoW2/DBoW2/BowVector.cpp, FeatureVector.cpp; oracle/ref_dbow2.mk) into
// oracle/_ref/.  These two files are the only part of the path that builds without
// OpenCV; TemplatedVocabulary.h (the tree walk) includes <opencv2/core/core.hpp> and does
// not.  The harness feeds the reference containers with per-feature (word, weight, node)
// triples and applies the frame-level steps of TemplatedVocabulary::transform
// (TemplatedVocabulary.h:1127-1186), so the oracle's BowVector / FeatureVector arithmetic
// -- accumulation order, the 1/size scaling, L1 / L2 normalisation -- is checked against
// the reference's compiled code (tests/test_vocab_ref.py).
#include <cstdint>

#include "BowVector.h"
#include "FeatureVector.h"

extern "C" {

// weighting: 0 TF_IDF, 1 TF, 2 IDF, 3 BINARY; scoring: 0 L1_NORM, 1 L2_NORM, 2 CHI_SQUARE,
// 3 KL, 4 BHATTACHARYYA, 5 DOT_PRODUCT (BowVector.h:36-53).  Outputs ascending by word /
// node (std::map order); returns the BowVector size, *nfv the FeatureVector's node count.
int dbow2_ref_frame(int n, const uint32_t* word, const double* weight, const uint32_t* node, int weighting,
                    int scoring, uint32_t* bow_word, double* bow_value, uint32_t* fv_node, int32_t* fv_off,
                    uint32_t* fv_idx, int* nfv) {
    DBoW2::BowVector v;
    DBoW2::FeatureVector fv;
    // ScoringObject.h:74-89: every scoring but DOT_PRODUCT normalises, L2 with L2_NORM
    const bool must = scoring != 5;
    const DBoW2::LNorm norm = scoring == 1 ? DBoW2::L2 : DBoW2::L1;
    const bool tf = weighting == 0 || weighting == 1;
    for (int i = 0; i < n; i++) {
        if (weight[i] > 0) {  // not stopped
            if (tf)
                v.addWeight(word[i], weight[i]);
            else
                v.addIfNotExist(word[i], weight[i]);
            fv.addFeature(node[i], (unsigned)i);
        }
    }
    if (tf && !v.empty() && !must) {
        const double nd = v.size();
        for (DBoW2::BowVector::iterator vit = v.begin(); vit != v.end(); vit++) vit->second /= nd;
    }
    if (must) v.normalize(norm);
    int k = 0;
    for (const auto& e : v) {
        bow_word[k] = e.first;
        bow_value[k] = e.second;
        k++;
    }
    int j = 0, o = 0;
    for (const auto& e : fv) {
        fv_node[j] = e.first;
        fv_off[j] = o;
        for (unsigned idx : e.second) fv_idx[o++] = idx;
        j++;
    }
    fv_off[j] = o;
    *nfv = j;
    return k;
}
}
