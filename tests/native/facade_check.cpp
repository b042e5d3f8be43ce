// Compile-and-run check of the C++ facade (include/orb_slam_gpu.hpp) without a GPU:
// bad parameters throw, DescriptorDistance works, POD types line up with cv::KeyPoint.
#include <cstdio>
#include <cstring>
#include <vector>

#include "../../include/orb_slam_gpu.hpp"

int main() {
    static_assert(sizeof(orb_keypoint_t) == 28, "cv::KeyPoint layout");
    int fails = 0;
    try {
        ORB_SLAM::gpu::ORBextractor bad(0, 1.2f, 8);
        fails++;
    } catch (const std::runtime_error& e) {
        if (!std::strstr(e.what(), "status -22")) fails++;
    }
    uint8_t a[32] = {0}, b[32];
    std::memset(b, 0xFF, 32);
    if (ORB_SLAM::gpu::ORBmatcher::DescriptorDistance(a, b) != 256) fails++;
    b[0] = 0;
    if (ORB_SLAM::gpu::ORBmatcher::DescriptorDistance(a, b) != 248) fails++;
    // matcher family: argument validation happens before any device work
    orb_frame_view_t v{};
    v.nlevels = 0;  // invalid
    std::vector<int> out;
    try {
        ORB_SLAM::gpu::ORBmatcher(0.9f, true).WindowSearch(v, nullptr, v, 100, out);
        fails++;
    } catch (const std::runtime_error& e) {
        if (!std::strstr(e.what(), "status -22")) fails++;
    }
    std::printf("facade fails %d\n", fails);
    return fails;
}
