// orb_persist.hip — the reference's on-disk keyframe feature records (include/SaveLoadWorld.h),
// written and read on the host and packed on the device straight from extractor output.
//
// SaveWorldToFile (SaveLoadWorld.h:1254) writes, per keyframe, one record to each stream:
//   kfKeyPoints.bin / kfKeyPointsUn.bin (SaveLoadWorld.h:1406-1443)
//       0xEB 0x90 | size_t nKeys | nKeys x (x, y, size, angle, response : f32, octave, class_id : i32)
//   kfDescriptors.bin (SaveLoadWorld.h:1446-1460)
//       0xEB 0x90 | int nDes | nDes x 32 u8 (row-major descriptor rows)
// all little-endian as the x86-64 writer emits them (size_t 8 bytes, int 4).  LoadWroldFromFile
// reads them back (SaveLoadWorld.h:2098-2189): a wrong header is reported ("header error ...,
// shouldn't") and reading continues; a short stream sets the stream's fail bit per record.
// The keypoint record of a cv::KeyPoint is field-for-field orb_keypoint_t, so a record body is
// the keypoint array's bytes.
#include <hip/hip_runtime.h>

#include <cstring>
#include <string>

#include "../../include/orb_abi.h"
#include "orb_internal.h"

namespace {

constexpr uint8_t kHdr0 = 0xEB, kHdr1 = 0x90;  // saveHeader (SaveLoadWorld.h:1256)
constexpr size_t kKeyRec = 28, kDesRec = 32;

int perr(int code, const std::string& m) { return orb_internal_set_error(code, m); }

// Exclusive scan of the per-frame record sizes -> stream offsets (B + 1 entries), one
// workgroup: the records of frame b start where frame b-1's end, as the reference appends one
// keyframe after another.
__global__ void __launch_bounds__(1024) k_record_offsets(const int32_t* __restrict__ counts, int B,
                                                         int64_t* __restrict__ keyOff, int64_t* __restrict__ desOff) {
    __shared__ int64_t s_part[1024];
    const int tid = threadIdx.x;
    const int per = (B + 1023) / 1024;
    const int b0 = tid * per, b1 = min(b0 + per, B);
    int64_t sum = 0;
    for (int b = b0; b < b1; ++b) sum += counts[b];
    s_part[tid] = sum;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {  // inclusive Hillis-Steele scan of the partial sums
        const int64_t v = tid >= o ? s_part[tid - o] : 0;
        __syncthreads();
        s_part[tid] += v;
        __syncthreads();
    }
    int64_t run = tid ? s_part[tid - 1] : 0;  // keypoints before b0
    for (int b = b0; b < b1; ++b) {
        keyOff[b] = (int64_t)b * 10 + run * (int64_t)kKeyRec;
        desOff[b] = (int64_t)b * 6 + run * (int64_t)kDesRec;
        run += counts[b];
    }
    if (tid == 1023) {
        keyOff[B] = (int64_t)B * 10 + s_part[1023] * (int64_t)kKeyRec;
        desOff[B] = (int64_t)B * 6 + s_part[1023] * (int64_t)kDesRec;
    }
}

// One workgroup per frame: header + count, then the record bodies.  Stream offsets are even
// (header 2 + count 8 / 4, bodies multiples of 4), so the body is moved in 16-bit units: a
// keypoint body is 14 halfwords, a descriptor row 16.
__global__ void __launch_bounds__(256) k_pack_records(const orb_keypoint_t* __restrict__ kps,
                                                      const uint8_t* __restrict__ desc,
                                                      const int32_t* __restrict__ counts, int cap,
                                                      const int64_t* __restrict__ keyOff,
                                                      const int64_t* __restrict__ desOff, uint8_t* __restrict__ keys,
                                                      uint8_t* __restrict__ des) {
    const int b = blockIdx.x, tid = threadIdx.x;
    const int n = counts[b];
    uint8_t* K = keys + keyOff[b];
    uint8_t* D = des + desOff[b];
    if (tid == 0) {
        K[0] = kHdr0;
        K[1] = kHdr1;
        D[0] = kHdr0;
        D[1] = kHdr1;
    }
    if (tid < 4) {  // size_t nKeys (8 B LE) and int nDes (4 B LE), halfword by halfword
        const uint64_t nk = (uint64_t)(uint32_t)n;
        ((uint16_t*)(K + 2))[tid] = (uint16_t)(nk >> (16 * tid));
        if (tid < 2) ((uint16_t*)(D + 2))[tid] = (uint16_t)((uint32_t)n >> (16 * tid));
    }
    const uint16_t* ks = (const uint16_t*)(kps + (size_t)b * cap);
    uint16_t* kd = (uint16_t*)(K + 10);
    for (int i = tid; i < n * 14; i += 256) kd[i] = ks[i];
    const uint16_t* ds = (const uint16_t*)(desc + (size_t)b * cap * kDesRec);
    uint16_t* dd = (uint16_t*)(D + 6);
    for (int i = tid; i < n * 16; i += 256) dd[i] = ds[i];
}

}  // namespace

extern "C" {

size_t orb_keypoint_record_bytes(size_t n) { return 2 + sizeof(uint64_t) + kKeyRec * n; }

size_t orb_descriptor_record_bytes(int n) { return 2 + sizeof(int32_t) + kDesRec * (size_t)(n > 0 ? n : 0); }

int orb_write_keypoint_record(const orb_keypoint_t* kps, size_t n, uint8_t* out, size_t cap, size_t* written) {
    if ((n && !kps) || !out) return perr(ORB_EINVAL, "bad arguments");
    const size_t need = orb_keypoint_record_bytes(n);
    if (cap < need) return perr(ORB_ERANGE, "record buffer too small");
    out[0] = kHdr0;
    out[1] = kHdr1;
    const uint64_t nk = n;
    std::memcpy(out + 2, &nk, 8);
    if (n) std::memcpy(out + 10, kps, kKeyRec * n);
    if (written) *written = need;
    return ORB_OK;
}

int orb_read_keypoint_record(const uint8_t* in, size_t len, orb_keypoint_t* kps, size_t cap, size_t* n,
                             size_t* consumed, int* header_ok) {
    if (!in || !n) return perr(ORB_EINVAL, "bad arguments");
    if (len < 10) return perr(ORB_ERANGE, "truncated keypoint record (header / count)");
    if (header_ok) *header_ok = in[0] == kHdr0 && in[1] == kHdr1;  // reported, not fatal (SaveLoadWorld.h:2106-2107)
    uint64_t nk = 0;
    std::memcpy(&nk, in + 2, 8);
    if (nk > (len - 10) / kKeyRec) return perr(ORB_ERANGE, "truncated keypoint record (body)");
    *n = (size_t)nk;
    if (nk > cap) return perr(ORB_ERANGE, "keypoint capacity smaller than the record");
    if (nk && !kps) return perr(ORB_EINVAL, "bad arguments");
    if (nk) std::memcpy(kps, in + 10, kKeyRec * nk);
    if (consumed) *consumed = 10 + kKeyRec * nk;
    return ORB_OK;
}

int orb_write_descriptor_record(const uint8_t* desc, int n, uint8_t* out, size_t cap, size_t* written) {
    if (n < 0 || (n && !desc) || !out) return perr(ORB_EINVAL, "bad arguments");
    const size_t need = orb_descriptor_record_bytes(n);
    if (cap < need) return perr(ORB_ERANGE, "record buffer too small");
    out[0] = kHdr0;
    out[1] = kHdr1;
    const int32_t nd = n;
    std::memcpy(out + 2, &nd, 4);
    if (n) std::memcpy(out + 6, desc, kDesRec * (size_t)n);
    if (written) *written = need;
    return ORB_OK;
}

int orb_read_descriptor_record(const uint8_t* in, size_t len, uint8_t* desc, int cap, int* n, size_t* consumed,
                               int* header_ok) {
    if (!in || !n) return perr(ORB_EINVAL, "bad arguments");
    if (len < 6) return perr(ORB_ERANGE, "truncated descriptor record (header / count)");
    if (header_ok) *header_ok = in[0] == kHdr0 && in[1] == kHdr1;  // SaveLoadWorld.h:2171-2173
    int32_t nd = 0;
    std::memcpy(&nd, in + 2, 4);
    if (nd < 0) return perr(ORB_EINVAL, "negative descriptor count");
    if ((size_t)nd > (len - 6) / kDesRec) return perr(ORB_ERANGE, "truncated descriptor record (body)");
    *n = nd;
    if (nd > cap) return perr(ORB_ERANGE, "descriptor capacity smaller than the record");
    if (nd && !desc) return perr(ORB_EINVAL, "bad arguments");
    if (nd) std::memcpy(desc, in + 6, kDesRec * (size_t)nd);
    if (consumed) *consumed = 6 + kDesRec * (size_t)nd;
    return ORB_OK;
}

int orb_pack_keyframe_records_device(const orb_keypoint_t* d_kps, const uint8_t* d_desc, const int32_t* d_counts,
                                     int cap, int B, uint8_t* d_keys_stream, size_t keys_cap, uint8_t* d_des_stream,
                                     size_t des_cap, int64_t* d_key_offsets, int64_t* d_des_offsets, void* stream) {
    if (!d_kps || !d_desc || !d_counts || cap <= 0 || B < 0 || !d_keys_stream || !d_des_stream || !d_key_offsets ||
        !d_des_offsets)
        return perr(ORB_EINVAL, "bad arguments");
    if (B == 0) return ORB_OK;
    // worst case (every frame full): checkable without reading the counts back
    if (keys_cap < (size_t)B * orb_keypoint_record_bytes((size_t)cap) ||
        des_cap < (size_t)B * orb_descriptor_record_bytes(cap))
        return perr(ORB_ERANGE, "stream buffers smaller than B full records");
    if (((uintptr_t)d_keys_stream | (uintptr_t)d_des_stream | (uintptr_t)d_kps | (uintptr_t)d_desc) & 1u)
        return perr(ORB_EINVAL, "buffers must be 2-byte aligned");
    hipStream_t st = (hipStream_t)stream;
    hipLaunchKernelGGL(k_record_offsets, dim3(1), dim3(1024), 0, st, d_counts, B, d_key_offsets, d_des_offsets);
    hipLaunchKernelGGL(k_pack_records, dim3(B), dim3(256), 0, st, d_kps, d_desc, d_counts, cap, d_key_offsets,
                       d_des_offsets, d_keys_stream, d_des_stream);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return perr(ORB_EDEVICE, std::string("k_pack_records: ") + hipGetErrorString(e));
    return ORB_OK;
}

}  // extern "C"
