// orbx.hpp -- header-only C++ mirror of ORB_SLAM2::ORBextractor / ORBmatcher over the
// C ABI in orbx.h (liborbx.so).  Same class names, constructor arguments, call operator,
// getters and search entry points as include/ORBextractor.h:76-220 and
// include/ORBmatcher.h:47-228 of the reference, with OpenCV types replaced by plain
// containers (cv::KeyPoint == orbx_keypoint, 28 bytes; descriptor rows of 32 bytes).
// Errors throw orbx::Error on this side of the boundary; nothing throws across it.
#pragma once

#include <cstdint>
#include <stdexcept>
#include <string>
#include <vector>

#include "orbx.h"

namespace orbx {

struct Error : std::runtime_error {
    int code;
    Error(int c, const std::string& what) : std::runtime_error(what), code(c) {}
};

inline void check(int rc) {
    if (rc != ORBX_OK && rc != ORBX_EMPTY) throw Error(rc, std::string("orbx: ") + orbx_last_error());
}

class ORBextractor {
public:
    enum { HARRIS_SCORE = 0, FAST_SCORE = 1 };

    ORBextractor(int nfeatures, float scaleFactor, int nlevels, int iniThFAST, int minThFAST, int device = 0)
        : nlevels_(nlevels), scaleFactor_(scaleFactor) {
        orbx_extractor_params p{nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST};
        check(orbx_extractor_create(&p, device, &h_));
    }
    ~ORBextractor() { orbx_extractor_destroy(h_); }
    ORBextractor(const ORBextractor&) = delete;
    ORBextractor& operator=(const ORBextractor&) = delete;

    // operator()(image, mask, keypoints, descriptors): an empty image leaves the outputs
    // untouched (ORBextractor.cc:1517-1518); zero keypoints empty the descriptors.
    void operator()(const uint8_t* img, int width, int height, size_t stride, std::vector<orbx_keypoint>& keypoints,
                    std::vector<uint8_t>& descriptors) {
        if (!img || width <= 0 || height <= 0) return;
        int cap = 0;
        check(orbx_extractor_max_keypoints(h_, width, height, &cap));
        keypoints.resize((size_t)cap);
        descriptors.resize((size_t)cap * 32);
        int n = 0;
        check(orbx_extract(h_, img, width, height, stride, keypoints.data(), descriptors.data(), cap, &n));
        keypoints.resize((size_t)n);
        descriptors.resize((size_t)n * 32);
    }

    int GetLevels() const { return nlevels_; }
    float GetScaleFactor() const { return scaleFactor_; }
    std::vector<float> GetScaleFactors() const { return levels(0); }
    std::vector<float> GetInverseScaleFactors() const { return levels(1); }
    std::vector<float> GetScaleSigmaSquares() const { return levels(2); }
    std::vector<float> GetInverseScaleSigmaSquares() const { return levels(3); }

    // mvImagePyramid[level] of the last call (ROI only), row-major w x h
    std::vector<uint8_t> ImagePyramidLevel(int level, int* w, int* h, int frame = 0) {
        check(orbx_pyramid_level(h_, frame, level, nullptr, 0, w, h));
        std::vector<uint8_t> out((size_t)(*w) * (*h));
        check(orbx_pyramid_level(h_, frame, level, out.data(), (size_t)*w, nullptr, nullptr));
        return out;
    }

    orbx_extractor* handle() { return h_; }

private:
    std::vector<float> levels(int which) const {
        std::vector<float> a(nlevels_), b(nlevels_), c(nlevels_), d(nlevels_);
        check(orbx_extractor_levels(h_, nullptr, a.data(), b.data(), c.data(), d.data()));
        return which == 0 ? a : which == 1 ? b : which == 2 ? c : d;
    }
    orbx_extractor* h_ = nullptr;
    int nlevels_;
    float scaleFactor_;
};

class ORBmatcher {
public:
    static const int TH_HIGH = 100;
    static const int TH_LOW = 50;
    static const int HISTO_LENGTH = 30;

    explicit ORBmatcher(float nnratio = 0.6f, bool checkOri = true, int device = 0) {
        check(orbx_matcher_create(device, nnratio, checkOri ? 1 : 0, &h_));
    }
    ~ORBmatcher() { orbx_matcher_destroy(h_); }
    ORBmatcher(const ORBmatcher&) = delete;
    ORBmatcher& operator=(const ORBmatcher&) = delete;

    static int DescriptorDistance(const uint8_t* a, const uint8_t* b) { return orbx_hamming(a, b); }

    // SearchByProjection(Frame&, const vector<MapPoint*>&, th)
    int SearchByProjection(const orbx_frame_view& F, int32_t* mvpMapPoints, const std::vector<int32_t>& vpMapPoints,
                           const orbx_mappoints& mps, const orbx_track& trk, float th = 3) {
        int n = 0;
        check(orbx_search_by_projection_local(h_, &F, mvpMapPoints, vpMapPoints.data(), (int)vpMapPoints.size(), &mps,
                                              &trk, th, &n));
        return n;
    }

    // SearchByProjection(Frame& CurrentFrame, const Frame& LastFrame, th, bMono)
    int SearchByProjection(const orbx_frame_view& CurrentFrame, int32_t* curMapPoints, const orbx_frame_view& LastFrame,
                           const int32_t* lastMapPoints, const uint8_t* lastOutlier, const orbx_mappoints& mps,
                           float th, bool bMono) {
        int n = 0;
        check(orbx_search_by_projection_frame(h_, &CurrentFrame, curMapPoints, &LastFrame, lastMapPoints, lastOutlier,
                                              &mps, th, bMono ? 1 : 0, &n));
        return n;
    }

    // SearchByProjection(Frame& CurrentFrame, KeyFrame* pKF, const set<MapPoint*>& sAlreadyFound, th, ORBdist)
    int SearchByProjection(const orbx_frame_view& CurrentFrame, int32_t* curMapPoints, const orbx_frame_view& KF,
                           const int32_t* kfMapPoints, const uint8_t* alreadyFound, const orbx_mappoints& mps,
                           float th, int ORBdist) {
        int n = 0;
        check(orbx_search_by_projection_keyframe(h_, &CurrentFrame, curMapPoints, &KF, kfMapPoints, alreadyFound, &mps,
                                                 th, ORBdist, &n));
        return n;
    }

    // SearchByProjection(KeyFrame* pKF, cv::Mat Scw, const vector<MapPoint*>& vpPoints, vector<MapPoint*>& vpMatched, th)
    int SearchByProjection(const orbx_frame_view& KF, const float Scw[12], const std::vector<int32_t>& vpPoints,
                           int32_t* vpMatched, const orbx_mappoints& mps, int th) {
        int n = 0;
        check(orbx_search_by_projection_sim3(h_, &KF, Scw, vpPoints.data(), (int)vpPoints.size(), vpMatched, &mps, th,
                                             &n));
        return n;
    }

    // SearchForTriangulation(pKF1, pKF2, F12, vMatchedPairs, bOnlyStereo)
    struct FeatureVector {
        std::vector<int32_t> node, off, idx;  // CSR of DBoW2::FeatureVector
    };
    int SearchForTriangulation(const orbx_frame_view& KF1, const uint8_t* kf1HasMP, const FeatureVector& fv1,
                               const orbx_frame_view& KF2, const uint8_t* kf2HasMP, const FeatureVector& fv2,
                               const float F12[9], std::vector<std::pair<size_t, size_t>>& vMatchedPairs,
                               bool bOnlyStereo) {
        std::vector<int32_t> pairs((size_t)KF1.n * 2 + 2);
        int np = 0;
        check(orbx_search_for_triangulation(h_, &KF1, kf1HasMP, fv1.node.data(), fv1.off.data(), fv1.idx.data(),
                                            (int)fv1.node.size(), &KF2, kf2HasMP, fv2.node.data(), fv2.off.data(),
                                            fv2.idx.data(), (int)fv2.node.size(), F12, bOnlyStereo ? 1 : 0,
                                            pairs.data(), &np));
        vMatchedPairs.clear();
        for (int i = 0; i < np; i++) vMatchedPairs.emplace_back((size_t)pairs[2 * i], (size_t)pairs[2 * i + 1]);
        return np;
    }

    // SearchByBoW(KeyFrame* pKF, Frame& F, vector<MapPoint*>& vpMapPointMatches); kfMapPoints: id or -1
    int SearchByBoW(const orbx_frame_view& KF, const int32_t* kfMapPoints, const FeatureVector& kfFeatVec,
                    const orbx_frame_view& F, const FeatureVector& fFeatVec, std::vector<int32_t>& vpMapPointMatches) {
        vpMapPointMatches.assign((size_t)F.n, -1);
        int n = 0;
        check(orbx_search_by_bow_frame(h_, &KF, kfMapPoints, kfFeatVec.node.data(), kfFeatVec.off.data(),
                                       kfFeatVec.idx.data(), (int)kfFeatVec.node.size(), &F, fFeatVec.node.data(),
                                       fFeatVec.off.data(), fFeatVec.idx.data(), (int)fFeatVec.node.size(),
                                       vpMapPointMatches.data(), &n));
        return n;
    }

    // SearchByBoW(KeyFrame* pKF1, KeyFrame* pKF2, vector<MapPoint*>& vpMatches12)
    int SearchByBoW(const orbx_frame_view& KF1, const int32_t* mapPoints1, const FeatureVector& fv1,
                    const orbx_frame_view& KF2, const int32_t* mapPoints2, const FeatureVector& fv2,
                    std::vector<int32_t>& vpMatches12) {
        vpMatches12.assign((size_t)KF1.n, -1);
        int n = 0;
        check(orbx_search_by_bow_keyframes(h_, &KF1, mapPoints1, fv1.node.data(), fv1.off.data(), fv1.idx.data(),
                                           (int)fv1.node.size(), &KF2, mapPoints2, fv2.node.data(), fv2.off.data(),
                                           fv2.idx.data(), (int)fv2.node.size(), vpMatches12.data(), &n));
        return n;
    }

    // SearchForInitialization(F1, F2, vbPrevMatched, vnMatches12, windowSize); vbPrevMatched as x,y pairs
    int SearchForInitialization(const orbx_frame_view& F1, const orbx_frame_view& F2, std::vector<float>& vbPrevMatched,
                                std::vector<int>& vnMatches12, int windowSize = 10) {
        vnMatches12.assign((size_t)F1.n, -1);
        int n = 0;
        check(orbx_search_for_initialization(h_, &F1, &F2, vbPrevMatched.data(), vnMatches12.data(), windowSize, &n));
        return n;
    }

    // Fuse(KeyFrame* pKF, const vector<MapPoint*>& vpMapPoints, th): search part, best[k] = KF keypoint or -1
    void Fuse(const orbx_frame_view& KF, const std::vector<int32_t>& vpMapPoints, const uint8_t* skip,
              const orbx_mappoints& mps, std::vector<int32_t>& best, float th = 3.0f) {
        best.assign(vpMapPoints.size(), -1);
        check(orbx_fuse(h_, &KF, vpMapPoints.data(), (int)vpMapPoints.size(), skip, &mps, th, best.data()));
    }

    // Fuse(KeyFrame* pKF, cv::Mat Scw, vpPoints, th, vpReplacePoint): search part
    void Fuse(const orbx_frame_view& KF, const float Scw[12], const std::vector<int32_t>& vpPoints, const uint8_t* skip,
              const orbx_mappoints& mps, std::vector<int32_t>& best, float th = 4.0f) {
        best.assign(vpPoints.size(), -1);
        check(orbx_fuse_sim3(h_, &KF, Scw, vpPoints.data(), (int)vpPoints.size(), skip, &mps, th, best.data()));
    }

    // SearchBySim3(pKF1, pKF2, vpMatches12, s12, R12, t12, th)
    int SearchBySim3(const orbx_frame_view& KF1, const int32_t* mapPoints1, const uint8_t* alreadyMatched1,
                     const orbx_frame_view& KF2, const int32_t* mapPoints2, const uint8_t* alreadyMatched2,
                     const orbx_mappoints& mps, float s12, const float R12[9], const float t12[3], float th,
                     int32_t* vpMatches12) {
        int n = 0;
        check(orbx_search_by_sim3(h_, &KF1, mapPoints1, alreadyMatched1, &KF2, mapPoints2, alreadyMatched2, &mps, s12,
                                  R12, t12, th, vpMatches12, &n));
        return n;
    }

    orbx_matcher* handle() { return h_; }

private:
    orbx_matcher* h_ = nullptr;
};

// The RGB-D Frame constructor's steps after ExtractORB (Frame.cc:192-264, 227-230):
// UndistortKeyPoints (Frame.cc:586-628) and ComputeStereoFromRGBD (Frame.cc:888-909) over
// the depth image as GrabImageRGBD receives it -- ORBX_DEPTH_U16 (the library applies
// mDepthMapFactor, Tracking.cc:265-271) or ORBX_DEPTH_F32 -- with mDepthMapFactor =
// 1 / DepthMapFactor (Tracking.cc:166-170) and mbf.  mvuRight / mvDepth are -1 where the
// depth is not positive, as the reference's vectors are initialised.
inline void ComputeStereoFromRGBD(const orbx_camera& cam, const std::vector<orbx_keypoint>& mvKeys,
                                  const void* depth, int depthType, int width, int height, size_t rowBytes,
                                  float mDepthMapFactor, float mbf, std::vector<orbx_keypoint>& mvKeysUn,
                                  std::vector<float>& mvuRight, std::vector<float>& mvDepth, int device = 0) {
    const int n = (int)mvKeys.size();
    mvKeysUn.resize((size_t)n);
    mvuRight.assign((size_t)n, -1.0f);
    mvDepth.assign((size_t)n, -1.0f);
    check(orbx_compute_stereo_from_rgbd(device, &cam, mvKeys.data(), n, depth, depthType, width, height, rowBytes,
                                        mDepthMapFactor, mbf, mvKeysUn.data(), mvuRight.data(), mvDepth.data()));
}

}  // namespace orbx
