// nth_select.h — exact replay of libstdc++'s std::nth_element (GCC 11,
// /usr/include/c++/11/bits/stl_algo.h:1964-1986 __introselect; 75-97 __move_median_to_first;
// 1878-1906 __unguarded_partition[_pivot]; 1819-1849 insertion sort; 1642-1650 __heap_select;
// stl_heap.h:134-146, 223-265, 339-360 heap helpers).
//
// The reference's KeyPointsFilter::retainBest (OpenCV 2.4) calls
//   std::nth_element(kps.begin(), kps.begin() + n, kps.end(), response greater)
// and ORB-SLAM keeps the first n (ORBextractor.cc:683-685, 697-700).  Keypoint order and,
// under the many FAST score ties, keypoint identity both depend on the exact permutation,
// so this is a statement-for-statement restatement over an array of POD elements.  Every
// element carries its identity (packed position) in the bits the comparator ignores.
//
// Usable from host (unit-tested against std::nth_element) and device (one lane per list).
#ifndef ORB_NTH_SELECT_H
#define ORB_NTH_SELECT_H

#include <stdint.h>

#if defined(__HIPCC__)
#define ORB_HD __host__ __device__
#else
#define ORB_HD
#endif

namespace orbsel {

template <class T>
ORB_HD inline void swap_at(T* a, int i, int j) {
    T t = a[i];
    a[i] = a[j];
    a[j] = t;
}

template <class T, class Greater>
ORB_HD inline void move_median_to_first(T* a, int result, int x, int y, int z, Greater comp) {
    if (comp(a[x], a[y])) {
        if (comp(a[y], a[z]))
            swap_at(a, result, y);
        else if (comp(a[x], a[z]))
            swap_at(a, result, z);
        else
            swap_at(a, result, x);
    } else if (comp(a[x], a[z]))
        swap_at(a, result, x);
    else if (comp(a[y], a[z]))
        swap_at(a, result, z);
    else
        swap_at(a, result, y);
}

template <class T, class Greater>
ORB_HD inline int unguarded_partition(T* a, int first, int last, int pivot, Greater comp) {
    while (true) {
        while (comp(a[first], a[pivot])) ++first;
        --last;
        while (comp(a[pivot], a[last])) --last;
        if (!(first < last)) return first;
        swap_at(a, first, last);
        ++first;
    }
}

template <class T, class Greater>
ORB_HD inline void push_heap(T* a, int first, int hole, int top, T value, Greater comp) {
    int parent = (hole - 1) / 2;
    while (hole > top && comp(a[first + parent], value)) {
        a[first + hole] = a[first + parent];
        hole = parent;
        parent = (hole - 1) / 2;
    }
    a[first + hole] = value;
}

template <class T, class Greater>
ORB_HD inline void adjust_heap(T* a, int first, int hole, int len, T value, Greater comp) {
    const int top = hole;
    int second = hole;
    while (second < (len - 1) / 2) {
        second = 2 * (second + 1);
        if (comp(a[first + second], a[first + second - 1])) second--;
        a[first + hole] = a[first + second];
        hole = second;
    }
    if ((len & 1) == 0 && second == (len - 2) / 2) {
        second = 2 * (second + 1);
        a[first + hole] = a[first + second - 1];
        hole = second - 1;
    }
    push_heap(a, first, hole, top, value, comp);
}

template <class T, class Greater>
ORB_HD inline void heap_select(T* a, int first, int middle, int last, Greater comp) {
    const int len = middle - first;
    if (len >= 2) {  // __make_heap
        int parent = (len - 2) / 2;
        while (true) {
            T value = a[first + parent];
            adjust_heap(a, first, parent, len, value, comp);
            if (parent == 0) break;
            parent--;
        }
    }
    for (int i = middle; i < last; ++i)
        if (comp(a[i], a[first])) {  // __pop_heap(first, middle, i)
            T value = a[i];
            a[i] = a[first];
            adjust_heap(a, first, 0, len, value, comp);
        }
}

template <class T, class Greater>
ORB_HD inline void insertion_sort(T* a, int first, int last, Greater comp) {
    if (first == last) return;
    for (int i = first + 1; i != last; ++i) {
        if (comp(a[i], a[first])) {
            T val = a[i];
            for (int k = i; k > first; --k) a[k] = a[k - 1];  // move_backward
            a[first] = val;
        } else {  // __unguarded_linear_insert
            T val = a[i];
            int l = i, next = i - 1;
            while (comp(val, a[next])) {
                a[l] = a[next];
                l = next;
                --next;
            }
            a[l] = val;
        }
    }
}

ORB_HD inline int lg(int n) {  // std::__lg
    int r = 0;
    while (n > 1) {
        n >>= 1;
        ++r;
    }
    return r;
}

// std::nth_element(a, a + nth, a + n, comp)
template <class T, class Greater>
ORB_HD inline void introselect(T* a, int nth, int n, int depth, Greater comp) {
    int first = 0, last = n;
    while (last - first > 3) {
        if (depth == 0) {
            heap_select(a, first, nth + 1, last, comp);
            swap_at(a, first, nth);
            return;
        }
        --depth;
        int mid = first + (last - first) / 2;
        move_median_to_first(a, first, first + 1, mid, last - 1, comp);
        int cut = unguarded_partition(a, first + 1, last, first, comp);
        if (cut <= nth)
            first = cut;
        else
            last = cut;
    }
    insertion_sort(a, first, last, comp);
}

template <class T, class Greater>
ORB_HD inline void nth_element(T* a, int nth, int n, Greater comp) {
    if (n == 0 || nth == n) return;
    introselect(a, nth, n, lg(n) * 2, comp);
}

// KeyPointsFilter::retainBest(kps, n) + truncation: returns the kept count.
template <class T, class Greater>
ORB_HD inline int retain_best(T* a, int n, int keep, Greater comp) {
    if (n <= keep) return n;
    if (keep <= 0) return 0;
    nth_element(a, keep, n, comp);
    return keep;
}

#if defined(__HIPCC__)
// The same permutation computed by one wave (array and scratch in LDS).  libstdc++'s
// __unguarded_partition(lo, hi, pivot) advances a left cursor over elements comp(x, pivot) and
// a right cursor over comp(pivot, x), swapping where both stop.  Its k-th swap therefore
// exchanges L_k (the k-th left stopper from the left: !comp(a[p], pivot)) with R_k (the k-th
// right stopper from the right: !comp(pivot, a[p]); the pivot slot lo-1 is the last one) for
// as long as L_k < R_k, and it returns L_K when that lies below R_{K-1}, else R_{K-1} (the left
// cursor stops on the element the previous swap put there).  Positions in the untouched middle
// keep their original values, so the stopper lists of the original array decide everything:
// ballot-compacted lists, a ballot count of K, disjoint swaps.
// set bits of a ballot mask below the calling lane (v_mbcnt_lo / v_mbcnt_hi)
__device__ inline int lanes_below_wave(uint64_t m) {
    return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

template <class T, class Greater>
__device__ inline int unguarded_partition_wave(T* a, int lo, int hi, T pv, Greater comp, uint16_t* Lp, uint16_t* Rp,
                                               int lane) {
    int nl = 0, nr = 0;
    for (int c0 = lo; c0 < hi; c0 += 64) {
        const int p = c0 + lane;
        bool ls = false, rs = false;
        if (p < hi) {
            const T v = a[p];
            ls = !comp(v, pv);
            rs = !comp(pv, v);
        }
        const uint64_t mL = __ballot(ls), mR = __ballot(rs);
        if (ls) Lp[nl + lanes_below_wave(mL)] = (uint16_t)p;
        if (rs) Rp[nr + lanes_below_wave(mR)] = (uint16_t)p;
        nl += __popcll(mL);
        nr += __popcll(mR);
    }
    // R_k = Rp[nr - 1 - k] (k < nr), R_nr = lo - 1; L_k < R_k holds for a prefix k < K
    int K = 0;
    for (int k0 = 0; k0 < nl; k0 += 64) {
        const int k = k0 + lane;
        bool ok = false;
        if (k < nl) ok = (int)Lp[k] < (k < nr ? (int)Rp[nr - 1 - k] : lo - 1);
        const uint64_t m = __ballot(ok);
        K += __popcll(m);
        if (m != ~0ull) break;
    }
    for (int k = lane; k < K; k += 64) {
        const int l = Lp[k], r = k < nr ? (int)Rp[nr - 1 - k] : lo - 1;
        const T x = a[l], y = a[r];
        a[l] = y;
        a[r] = x;
    }
    const int LK = K < nl ? (int)Lp[K] : 0x7fffffff;
    const int Rprev = K == 0 ? hi : (K - 1 < nr ? (int)Rp[nr - K] : lo - 1);
    return LK < Rprev ? LK : Rprev;
}

// std::nth_element(a, a + nth, a + n, comp) by one wave of a workgroup (a, Lp, Rp in LDS;
// Lp / Rp hold n u16 each).  The median-of-3, the depth-limited heap fallback and the final
// insertion sort are the sequential code on lane 0; LDS accesses of one wave complete in
// order, so every lane sees lane 0's writes.
template <class T, class Greater>
__device__ inline void nth_element_wave(T* a, int nth, int n, Greater comp, uint16_t* Lp, uint16_t* Rp, int lane) {
    if (n == 0 || nth == n) return;
    int first = 0, last = n, depth = lg(n) * 2;
    while (last - first > 3) {
        if (depth == 0) {
            if (lane == 0) {
                heap_select(a, first, nth + 1, last, comp);
                swap_at(a, first, nth);
            }
            return;
        }
        --depth;
        const int mid = first + (last - first) / 2;
        if (lane == 0) move_median_to_first(a, first, first + 1, mid, last - 1, comp);
        const T pv = a[first];
        const int cut = unguarded_partition_wave(a, first + 1, last, pv, comp, Lp, Rp, lane);
        if (cut <= nth)
            first = cut;
        else
            last = cut;
    }
    if (lane == 0) insertion_sort(a, first, last, comp);
}

template <class T, class Greater>
__device__ inline int retain_best_wave(T* a, int n, int keep, Greater comp, uint16_t* Lp, uint16_t* Rp, int lane) {
    if (n <= keep) return n;
    if (keep <= 0) return 0;
    nth_element_wave(a, keep, n, comp, Lp, Rp, lane);
    return keep;
}
#endif

}  // namespace orbsel

#endif
