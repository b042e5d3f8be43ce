// orb_oracle_mappoint.cpp — TEST INFRASTRUCTURE ONLY (CPU parity checker; never linked by the product).
//
// MapPoint::ComputeDistinctiveDescriptors, reference src/MapPoint.cc:185-250, over flattened
// observations (rows offsets[m] .. offsets[m+1]-1 of desc, usable[r] = !pKF->isBad()), with the
// reference's own containers and arithmetic: float Distances[N][N], vector<int> rows sorted by
// std::sort, median = vDists[0.5*(N-1)], strict `median < BestMedian`.
#include <algorithm>
#include <climits>
#include <cstdint>
#include <cstring>
#include <vector>

#include "orb_oracle.h"

extern "C" int oracle_compute_distinctive_descriptors(int M, const int32_t* offsets, const uint8_t* desc,
                                                      const uint8_t* usable, int32_t* best_row, uint8_t* out_desc) {
    for (int m = 0; m < M; ++m) {
        std::vector<int> rows;  // vDescriptors (MapPoint.cc:202-210)
        for (int r = offsets[m]; r < offsets[m + 1]; ++r)
            if (!usable || usable[r]) rows.push_back(r);
        if (rows.empty()) {  // 212-213: mDescriptor unchanged
            best_row[m] = -1;
            continue;
        }
        const size_t N = rows.size();
        std::vector<float> Distances(N * N);  // float Distances[N][N] (218)
        for (size_t i = 0; i < N; i++) {
            Distances[i * N + i] = 0;
            for (size_t j = i + 1; j < N; j++) {
                const int distij = oracle_descriptor_distance(desc + 32 * (size_t)rows[i], desc + 32 * (size_t)rows[j]);
                Distances[i * N + j] = distij;
                Distances[j * N + i] = distij;
            }
        }
        int BestMedian = INT_MAX;
        int BestIdx = 0;
        for (size_t i = 0; i < N; i++) {
            std::vector<int> vDists(Distances.begin() + i * N, Distances.begin() + (i + 1) * N);
            std::sort(vDists.begin(), vDists.end());
            const int median = vDists[0.5 * (N - 1)];
            if (median < BestMedian) {
                BestMedian = median;
                BestIdx = (int)i;
            }
        }
        best_row[m] = rows[BestIdx];
        std::memcpy(out_desc + 32 * (size_t)m, desc + 32 * (size_t)rows[BestIdx], 32);
    }
    return 0;
}
