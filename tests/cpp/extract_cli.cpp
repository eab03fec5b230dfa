// Drives the C++ mirror (include/orbx.hpp) the way Frame::ExtractORB drives the
// reference ORBextractor (Frame.cc:377-386), then one ORBmatcher call.
//   extract_cli <raw u8 image> <width> <height> <out.bin>
// out.bin: int32 n, n x 28-byte keypoints, n x 32-byte descriptors.
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "orbx.hpp"

int main(int argc, char** argv) {
    if (argc != 5) {
        std::fprintf(stderr, "usage: %s img.raw W H out.bin\n", argv[0]);
        return 2;
    }
    const int W = std::atoi(argv[2]), H = std::atoi(argv[3]);
    std::vector<uint8_t> img((size_t)W * H);
    FILE* f = std::fopen(argv[1], "rb");
    if (!f || std::fread(img.data(), 1, img.size(), f) != img.size()) return 3;
    std::fclose(f);
    try {
        orbx::ORBextractor extractor(1000, 1.2f, 8, 20, 7);
        std::vector<orbx_keypoint> kps;
        std::vector<uint8_t> desc;
        extractor(img.data(), W, H, (size_t)W, kps, desc);
        if (extractor.GetLevels() != 8 || extractor.GetScaleFactors().size() != 8) return 4;
        const int d01 = kps.size() > 1 ? orbx::ORBmatcher::DescriptorDistance(&desc[0], &desc[32]) : 0;
        std::printf("n=%zu d01=%d\n", kps.size(), d01);
        FILE* o = std::fopen(argv[4], "wb");
        const int n = (int)kps.size();
        std::fwrite(&n, 4, 1, o);
        std::fwrite(kps.data(), sizeof(orbx_keypoint), kps.size(), o);
        std::fwrite(desc.data(), 1, desc.size(), o);
        std::fclose(o);
    } catch (const orbx::Error& e) {
        std::fprintf(stderr, "%s\n", e.what());
        return 1;
    }
    return 0;
}
