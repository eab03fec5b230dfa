// Drives the C++ mirror's RGB-D Frame step (include/orbx.hpp ComputeStereoFromRGBD) the way
// Frame's RGB-D constructor runs after ExtractORB (Frame.cc:217-230): extract a gray image,
// then undistort the keypoints and look their depth up in a 16-bit depth image.
//   rgbd_cli <gray u8> <depth u16> <W> <H> <fx fy cx cy k1 k2 p1 p2 k3> <DepthMapFactor> <bf> <out.bin>
// out.bin: int32 n, n x 28-byte keypoints, n x 28-byte undistorted keypoints, n floats
// mvuRight, n floats mvDepth.
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "orbx.hpp"

int main(int argc, char** argv) {
    if (argc != 17) {
        std::fprintf(stderr, "usage: %s gray.raw depth.raw W H fx fy cx cy k1 k2 p1 p2 k3 factor bf out.bin\n", argv[0]);
        return 2;
    }
    const int W = std::atoi(argv[3]), H = std::atoi(argv[4]);
    orbx_camera cam{};
    float* c = &cam.fx;
    for (int i = 0; i < 9; i++) c[i] = std::strtof(argv[5 + i], nullptr);
    const float factor = std::strtof(argv[14], nullptr), bf = std::strtof(argv[15], nullptr);
    std::vector<uint8_t> gray((size_t)W * H);
    std::vector<uint16_t> depth((size_t)W * H);
    FILE* f = std::fopen(argv[1], "rb");
    if (!f || std::fread(gray.data(), 1, gray.size(), f) != gray.size()) return 3;
    std::fclose(f);
    f = std::fopen(argv[2], "rb");
    if (!f || std::fread(depth.data(), 2, depth.size(), f) != depth.size()) return 3;
    std::fclose(f);
    try {
        orbx::ORBextractor extractor(5000, 1.2f, 12, 20, 7);
        std::vector<orbx_keypoint> kps, kpu;
        std::vector<uint8_t> desc;
        std::vector<float> ur, dp;
        extractor(gray.data(), W, H, (size_t)W, kps, desc);
        // Tracking.cc:166-170: mDepthMapFactor = 1 / DepthMapFactor
        const float mDepthMapFactor = factor == 0.0f ? 1.0f : 1.0f / factor;
        orbx::ComputeStereoFromRGBD(cam, kps, depth.data(), ORBX_DEPTH_U16, W, H, (size_t)W * 2, mDepthMapFactor, bf,
                                    kpu, ur, dp);
        FILE* o = std::fopen(argv[16], "wb");
        const int n = (int)kps.size();
        std::fwrite(&n, 4, 1, o);
        std::fwrite(kps.data(), sizeof(orbx_keypoint), kps.size(), o);
        std::fwrite(kpu.data(), sizeof(orbx_keypoint), kpu.size(), o);
        std::fwrite(ur.data(), 4, ur.size(), o);
        std::fwrite(dp.data(), 4, dp.size(), o);
        std::fclose(o);
        std::printf("n=%d\n", n);
    } catch (const orbx::Error& e) {
        std::fprintf(stderr, "%s\n", e.what());
        return 1;
    }
    return 0;
}
