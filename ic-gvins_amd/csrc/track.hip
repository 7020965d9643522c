// track.hip -- the glue kernels of gvx_track_frame_dev: one frame of
// Tracking::track's image path with the tracker state in device memory and every
// size read on the device, so a frame needs no host round trip and the launch
// topology is fixed (a hipGraph per frame replays it).  Paths under
// /root/reference/ic_gvins/ic_gvins/:
//   track_update_kernel  reduceVector of the FB result (tracking.cc:396-408,
//                        :831-839) and the next initial flow (pts + vel)
//   detect_prep_kernel   featuresDetection's early exit and per-block counts
//                        (tracking.cc:579-606), the circle centres of the
//                        tracked points (:617-619, cvRound), the active blocks
//   detect_merge_kernel  the corners in block order with the block origin
//                        (:669-685), appended up to track_max_features_
// They follow SequenceTracker (gvx/tracking.py), whose host arithmetic they
// replace: float32 next - pts, pts + vel, lrintf centres, int block indices.
#include <hip/hip_runtime.h>

#include "gvx_internal.h"

namespace gvx {

namespace {

constexpr int TU_THREADS = 256;

__device__ __forceinline__ void track_update(int cap, int32_t* __restrict__ n_ptr, const uint8_t* __restrict__ flags,
                                             const float2* __restrict__ next_xy, float2* __restrict__ pts,
                                             float2* __restrict__ vel, float2* __restrict__ init,
                                             int32_t* __restrict__ kept_out, int* wsum, int& base_s) {
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int n = min(*n_ptr, cap);
    int base = 0;
    // chunk by chunk: a kept point moves to an index <= its own, and every read of
    // a chunk happens before its writes (barrier), so the update is in place
    for (int start = 0; start < n; start += TU_THREADS) {
        const int i = start + tid;
        const bool k = i < n && (flags[i] & 4);
        const unsigned long long m = __ballot(k);
        const int before = __popcll(m & ((1ull << lane) - 1ull));
        if (lane == 0) wsum[wv] = __popcll(m);
        __syncthreads();
        int off = base;
        for (int w = 0; w < wv; ++w) off += wsum[w];
        int tot = 0;
        for (int w = 0; w < TU_THREADS / 64; ++w) tot += wsum[w];
        float2 nx{}, p{};
        if (k) {
            nx = next_xy[i];
            p = pts[i];
        }
        __syncthreads();
        if (k) {
            const int j = off + before;
            const float2 v = make_float2(nx.x - p.x, nx.y - p.y);
            pts[j] = nx;
            vel[j] = v;
            init[j] = make_float2(nx.x + v.x, nx.y + v.y);
            if (kept_out) kept_out[j] = i;
        }
        base += tot;
        __syncthreads();
    }
    if (tid == 0) base_s = base;
    __syncthreads();
    if (tid == 0) *n_ptr = base_s;
}

__global__ void __launch_bounds__(TU_THREADS) track_update_kernel(int cap, int32_t* __restrict__ n_ptr,
                                                                  const uint8_t* __restrict__ flags,
                                                                  const float2* __restrict__ next_xy,
                                                                  float2* __restrict__ pts, float2* __restrict__ vel,
                                                                  float2* __restrict__ init,
                                                                  int32_t* __restrict__ kept_out) {
    __shared__ int wsum[TU_THREADS / 64];
    __shared__ int base_s;
    track_update(cap, n_ptr, flags, next_xy, pts, vel, init, kept_out, wsum, base_s);
}

__global__ void __launch_bounds__(256) detect_prep_kernel(DetectPrep p) {
    __shared__ int cnt[1024];
    const int tid = threadIdx.x;
    if (p.update_cap > 0) {
        // the frame's reduceVector first (one launch instead of two; the writes
        // are visible to this workgroup after the barrier)
        __shared__ int wsum[TU_THREADS / 64];
        __shared__ int base_s;
        track_update(p.update_cap, p.n_upd, p.flags, reinterpret_cast<const float2*>(p.next_xy),
                     reinterpret_cast<float2*>(p.upd_pts), reinterpret_cast<float2*>(p.vel),
                     reinterpret_cast<float2*>(p.init), p.kept_out, wsum, base_s);
        __syncthreads();
    }
    const int bcnt = p.bcols * p.brows;
    const int n = *p.n;
    // featuresDetection is called while the tracks are below track_max_features_
    // (SequenceTracker: n < N) and returns early when n > track_max_features_ - 5
    const bool skip = !(n < p.max_features) || n > p.max_features - 5 || p.maxpb <= 0;
    for (int k = tid; k < bcnt; k += 256) {
        cnt[k] = 0;
        p.ncorner[k] = 0;
    }
    __syncthreads();
    if (!skip) {
        for (int i = tid; i < n; i += 256) {
            const float x = p.pts[2 * i], y = p.pts[2 * i + 1];
            const int cc = (int)(x / (float)p.col);
            const int rr = (int)(y / (float)p.row);
            const int idx = rr * p.bcols + cc;
            if (idx >= 0 && idx < bcnt) atomicAdd(&cnt[idx], 1);
            p.centers[i] = make_int2((int)rintf(x), (int)rintf(y));
        }
    }
    __syncthreads();
    if (tid == 0) {
        int na = 0;
        if (!skip)
            for (int k = 0; k < bcnt; ++k) {
                p.want[k] = p.maxpb - cnt[k];
                if (p.want[k] > 0) p.blk_ids[na++] = k;
            }
        *p.n_active = na;
        *p.n_circles = skip ? 0 : n;
        *p.skip = skip ? 1 : 0;
    }
}

// the detected corners in block order with the block origin, appended to the
// track list up to max_features (tracking.cc:669-685)
__device__ __forceinline__ void merge_corners(int bcnt, int bcols, int col, int row, int maxpb, int max_features,
                                              const int* __restrict__ ncorner, const float2* __restrict__ out,
                                              float2* __restrict__ pts, float2* __restrict__ vel,
                                              float2* __restrict__ init, int32_t* __restrict__ n_ptr,
                                              float2* __restrict__ corners_out, int32_t* __restrict__ n_corners_out,
                                              int* off) {
    const int tid = threadIdx.x;
    if (tid == 0) {
        int t = 0;
        for (int k = 0; k < bcnt; ++k) {
            off[k] = t;
            t += ncorner[k];
        }
        off[bcnt] = t;
    }
    __syncthreads();
    const int total = off[bcnt];
    const int n = *n_ptr;
    const int add = min(total, max_features - n);
    for (int k = 0; k < bcnt; ++k) {
        const int nc = ncorner[k];
        const int bc = k % bcols, br = k / bcols;
        for (int i = tid; i < nc; i += 256) {
            const float2 v = out[(int64_t)k * maxpb + i];
            const float2 c = make_float2((float)(bc * col) + v.x, (float)(br * row) + v.y);
            const int j = off[k] + i;
            if (corners_out) corners_out[j] = c;
            if (j < add) {
                pts[n + j] = c;
                vel[n + j] = make_float2(0.f, 0.f);
                init[n + j] = c;  // pts + vel with vel = 0
            }
        }
    }
    __syncthreads();
    if (tid == 0) {
        if (add > 0) *n_ptr = n + add;
        if (n_corners_out) *n_corners_out = total;
    }
}

__global__ void __launch_bounds__(256) detect_merge_kernel(int bcnt, int bcols, int col, int row, int maxpb,
                                                           int max_features, const int* __restrict__ skip,
                                                           const int* __restrict__ ncorner,
                                                           const float2* __restrict__ out, float2* __restrict__ pts,
                                                           float2* __restrict__ vel, float2* __restrict__ init,
                                                           int32_t* __restrict__ n_ptr, float2* __restrict__ corners_out,
                                                           int32_t* __restrict__ n_corners_out, TrackRecord rec) {
    __shared__ int off[1025];
    const int tid = threadIdx.x;
    if (*skip) {  // wave-uniform (one value for the launch)
        if (tid == 0 && n_corners_out) *n_corners_out = -1;
    } else {
        merge_corners(bcnt, bcols, col, row, maxpb, max_features, ncorner, out, pts, vel, init, n_ptr, corners_out,
                      n_corners_out, off);
    }
    if (rec.tracks) {
        // the track list appended to the per-frame record at *rec.frame, which
        // advances (launch_track_record, fused: one launch less per frame)
        __syncthreads();  // the merged list (pts, *n_ptr) is visible to the workgroup
        const int f = *rec.frame;
        const int n = min(*n_ptr, rec.cap);
        if (f < rec.max_frames) {
            for (int i = tid; i < n; i += 256) reinterpret_cast<float2*>(rec.tracks)[(int64_t)f * rec.cap + i] = pts[i];
            if (tid == 0) rec.counts[f] = n;
        }
        __syncthreads();
        if (tid == 0) *rec.frame = f + 1;
    }
}

// The tracking path's last launch (after select_track_kernel): the frame's
// reduceVector of the FB result (track frames), featuresDetection's early exit
// recomputed from the kept count (the selection workgroups took the same
// decision), the corners appended, and the per-frame record.
__global__ void __launch_bounds__(256) track_merge_kernel(TrackMerge m) {
    __shared__ int wsum[TU_THREADS / 64];
    __shared__ int base_s;
    __shared__ int off[1025];
    const int tid = threadIdx.x;
    if (m.update_cap > 0) {
        track_update(m.update_cap, m.n, m.flags, reinterpret_cast<const float2*>(m.next_xy),
                     reinterpret_cast<float2*>(m.pts), reinterpret_cast<float2*>(m.vel),
                     reinterpret_cast<float2*>(m.init), m.kept_out, wsum, base_s);
        __syncthreads();
    }
    const int n = *m.n;
    const bool skip = !(n < m.max_features) || n > m.max_features - 5 || m.maxpb <= 0;
    if (skip) {
        if (tid == 0 && m.n_corners_out) *m.n_corners_out = -1;
    } else {
        merge_corners(m.bcnt, m.bcols, m.col, m.row, m.out_stride, m.max_features, m.ncorner, m.out,
                      reinterpret_cast<float2*>(m.pts), reinterpret_cast<float2*>(m.vel),
                      reinterpret_cast<float2*>(m.init), m.n, reinterpret_cast<float2*>(m.corners_out),
                      m.n_corners_out, off);
    }
    if (m.rec.tracks) {
        __syncthreads();
        const int f = *m.rec.frame;
        const int nn = min(*m.n, m.rec.cap);
        if (f < m.rec.max_frames) {
            for (int i = tid; i < nn; i += 256)
                reinterpret_cast<float2*>(m.rec.tracks)[(int64_t)f * m.rec.cap + i] = reinterpret_cast<const float2*>(m.pts)[i];
            if (tid == 0) m.rec.counts[f] = nn;
        }
        __syncthreads();
        if (tid == 0) *m.rec.frame = f + 1;
    }
}

// gvx_copy_dev as a kernel: a copy node on the compute queue instead of a DMA
// copy (in a captured graph the memcpy node cost more than the pair's kernels)
__global__ void __launch_bounds__(256) copy_kernel(uint8_t* __restrict__ dst, const uint8_t* __restrict__ src,
                                                   size_t bytes) {
    const size_t stride = (size_t)gridDim.x * 256;
    size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if ((((uintptr_t)dst | (uintptr_t)src) & 15) == 0) {
        const size_t n16 = bytes >> 4;
        for (size_t k = i; k < n16; k += stride)
            reinterpret_cast<uint4*>(dst)[k] = reinterpret_cast<const uint4*>(src)[k];
        for (size_t k = (n16 << 4) + i; k < bytes; k += stride) dst[k] = src[k];
    } else {
        for (size_t k = i; k < bytes; k += stride) dst[k] = src[k];
    }
}

// dst <- src_base + (*index) * bytes: a copy whose source is chosen on the device
__global__ void __launch_bounds__(256) copy_indexed_kernel(uint8_t* __restrict__ dst,
                                                           const uint8_t* __restrict__ src_base, size_t bytes,
                                                           const int32_t* __restrict__ index, int n_src) {
    const uint8_t* src = src_base + (size_t)min(max(*index, 0), n_src - 1) * bytes;
    const size_t stride = (size_t)gridDim.x * 256;
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if ((((uintptr_t)dst | (uintptr_t)src) & 15) == 0) {
        const size_t n16 = bytes >> 4;
        for (size_t k = i; k < n16; k += stride)
            reinterpret_cast<uint4*>(dst)[k] = reinterpret_cast<const uint4*>(src)[k];
        for (size_t k = (n16 << 4) + i; k < bytes; k += stride) dst[k] = src[k];
    } else {
        for (size_t k = i; k < bytes; k += stride) dst[k] = src[k];
    }
}

// the current track list appended to a per-frame record at a device-held frame
// index, which then advances (frames beyond max_frames are dropped)
__global__ void __launch_bounds__(256) track_record_kernel(const float2* __restrict__ pts,
                                                           const int32_t* __restrict__ n_ptr, int cap,
                                                           float2* __restrict__ tracks, int32_t* __restrict__ counts,
                                                           int32_t* __restrict__ frame, int max_frames) {
    const int f = *frame;
    const int n = min(*n_ptr, cap);
    if (f < max_frames) {
        for (int i = threadIdx.x; i < n; i += 256) tracks[(int64_t)f * cap + i] = pts[i];
        if (threadIdx.x == 0) counts[f] = n;
    }
    __syncthreads();
    if (threadIdx.x == 0) *frame = f + 1;
}

}  // namespace

// *index += delta (a frame counter a graph advances for itself)
__global__ void __launch_bounds__(64) index_advance_kernel(int32_t* __restrict__ index, int32_t delta) {
    if (threadIdx.x == 0) index[0] += delta;
}

hipError_t launch_index_advance(gvx_ctx* c, int32_t* index, int32_t delta) {
    index_advance_kernel<<<1, 64, 0, c->stream>>>(index, delta);
    return hipGetLastError();
}

hipError_t launch_copy_indexed(gvx_ctx* c, void* dst, const void* src_base, size_t bytes, const int32_t* index,
                               int n_src) {
    const size_t units = (bytes + 15) / 16;
    const unsigned blocks = (unsigned)std::min<size_t>((units + 255) / 256, 4096);
    copy_indexed_kernel<<<blocks ? blocks : 1, 256, 0, c->stream>>>(static_cast<uint8_t*>(dst),
                                                                    static_cast<const uint8_t*>(src_base), bytes,
                                                                    index, n_src);
    return hipGetLastError();
}

hipError_t launch_track_record(gvx_ctx* c, const float* pts, const int32_t* n, int cap, float* tracks,
                               int32_t* counts, int32_t* frame, int max_frames) {
    track_record_kernel<<<1, 256, 0, c->stream>>>(reinterpret_cast<const float2*>(pts), n, cap,
                                                  reinterpret_cast<float2*>(tracks), counts, frame, max_frames);
    return hipGetLastError();
}

hipError_t launch_copy(gvx_ctx* c, void* dst, const void* src, size_t bytes) {
    const size_t units = (bytes + 15) / 16;
    const unsigned blocks = (unsigned)std::min<size_t>((units + 255) / 256, 4096);
    copy_kernel<<<blocks ? blocks : 1, 256, 0, c->stream>>>(static_cast<uint8_t*>(dst),
                                                            static_cast<const uint8_t*>(src), bytes);
    return hipGetLastError();
}

hipError_t launch_track_update(gvx_ctx* c, int cap, int32_t* n, const uint8_t* flags, const float* next_xy,
                               float* pts, float* vel, float* init, int32_t* kept_out) {
    track_update_kernel<<<1, TU_THREADS, 0, c->stream>>>(cap, n, flags, reinterpret_cast<const float2*>(next_xy),
                                                         reinterpret_cast<float2*>(pts), reinterpret_cast<float2*>(vel),
                                                         reinterpret_cast<float2*>(init), kept_out);
    return hipGetLastError();
}

hipError_t launch_detect_prep(gvx_ctx* c, const DetectPrep& p) {
    if (p.bcols * p.brows > 1024) return hipErrorInvalidValue;
    detect_prep_kernel<<<1, 256, 0, c->stream>>>(p);
    return hipGetLastError();
}

hipError_t launch_track_merge(gvx_ctx* c, const TrackMerge& m) {
    if (m.bcnt > 1024) return hipErrorInvalidValue;
    track_merge_kernel<<<1, 256, 0, c->stream>>>(m);
    return hipGetLastError();
}

hipError_t launch_detect_merge(gvx_ctx* c, int bcnt, int bcols, int col, int row, int maxpb, int max_features,
                               const int* skip, const int* ncorner, const float2* out, float* pts, float* vel,
                               float* init, int32_t* n, float* corners_out, int32_t* n_corners_out,
                               const TrackRecord* rec) {
    if (bcnt > 1024) return hipErrorInvalidValue;
    const TrackRecord r = rec ? *rec : TrackRecord{};
    detect_merge_kernel<<<1, 256, 0, c->stream>>>(bcnt, bcols, col, row, maxpb, max_features, skip, ncorner, out,
                                                  reinterpret_cast<float2*>(pts), reinterpret_cast<float2*>(vel),
                                                  reinterpret_cast<float2*>(init), n,
                                                  reinterpret_cast<float2*>(corners_out), n_corners_out, r);
    return hipGetLastError();
}

}  // namespace gvx
