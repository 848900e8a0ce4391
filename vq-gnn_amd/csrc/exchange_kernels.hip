// Multi-GPU code exchange wire format (no counterpart in the single-process
// reference; keeps every replica's c_indices — models.py:46/:63 — identical).
//
// One record per batch row: int32 node id (-1 = padding) followed by the row's
// nb codes as uint8 (M <= 256) or int16, padded to a multiple of 4 bytes.  A
// rank packs its rows (and scatters them into its own c_indices at once), one
// all_gather_into_tensor moves the records, and every rank scatters all of
// them with "the last record wins" for a node several ranks hold — the order
// of the union batch on one GPU (index_put with repeated indices writes in
// order on the CPU).  The winner is chosen deterministically (an atomicMax of
// the stamp epoch << 32 | record index per node, then only the winner
// writes), so every replica resolves repeats the same way.  The epoch grows
// with every exchange, so stamps of earlier exchanges are smaller than any of
// this one and the table is never reset: no pass, no lane, no wave ever
// writes it except the atomicMax (a reset by the winner lane raced with the
// other lanes of the same record when they sat in another wave).

#include "common.h"

namespace vqgnn {

__host__ __device__ inline int wire_code_bytes(int M) { return M <= 256 ? 1 : 2; }
__host__ __device__ inline int wire_record_bytes(int nb, int M) {
  return (4 + nb * wire_code_bytes(M) + 3) / 4 * 4;
}

// one thread per row; the common shape (uint8 wire, nb % 4 == 0, aligned
// rows) moves whole words: 8-byte reads of 4 codes, 4-byte record writes
__global__ void pack_codes_kernel(const int64_t* __restrict__ batch_idx, int B,
                                  const int16_t* __restrict__ local, int nb, int M, int max_B,
                                  uint8_t* __restrict__ send, int16_t* __restrict__ codes,
                                  int64_t ldc, int vec) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= max_B) return;
  const int rec = wire_record_bytes(nb, M);
  uint8_t* p = send + (int64_t)r * rec;
  if (r >= B) {
    *reinterpret_cast<int32_t*>(p) = -1;
    return;
  }
  const int64_t node = batch_idx[r];
  *reinterpret_cast<int32_t*>(p) = (int32_t)node;
  const int16_t* l = local + (int64_t)r * nb;
  int16_t* c = (codes && node >= 0) ? codes + node * ldc : nullptr;
  if (vec) {
    uint32_t* pw = reinterpret_cast<uint32_t*>(p + 4);
    for (int b = 0; b < nb; b += 4) {
      const uint2 t = *reinterpret_cast<const uint2*>(l + b);   // 4 int16 codes
      pw[b / 4] = (t.x & 0xFFu) | ((t.x >> 16 & 0xFFu) << 8) | ((t.y & 0xFFu) << 16) |
                  ((t.y >> 16 & 0xFFu) << 24);
      if (c) *reinterpret_cast<uint2*>(c + b) = t;
    }
    return;
  }
  if (wire_code_bytes(M) == 1) {
    for (int b = 0; b < nb; ++b) p[4 + b] = (uint8_t)l[b];
  } else {
    int16_t* q = reinterpret_cast<int16_t*>(p + 4);
    for (int b = 0; b < nb; ++b) q[b] = l[b];
  }
  if (c)
    for (int b = 0; b < nb; ++b) c[b] = l[b];
}

// Eight codes per thread (uint8 wire, 8 | nb, 16-byte aligned code rows):
// thread (row, chunk) reads one 16-byte piece of the row's int16 codes,
// writes 8 wire bytes and (own rows) the 16-byte piece of c_indices.
__global__ void pack_codes8_kernel(const int64_t* __restrict__ batch_idx, int B,
                                   const int16_t* __restrict__ local, int nb, int max_B,
                                   uint8_t* __restrict__ send, int16_t* __restrict__ codes,
                                   int64_t ldc) {
  const int ch = nb >> 3;
  const int64_t tix = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (tix >= (int64_t)max_B * ch) return;
  const int r = (int)(tix / ch), c = (int)(tix % ch);
  const int rec = wire_record_bytes(nb, 256);
  uint8_t* p = send + (int64_t)r * rec;
  if (r >= B) {
    if (c == 0) *reinterpret_cast<int32_t*>(p) = -1;
    return;
  }
  const int64_t node = batch_idx[r];
  if (c == 0) *reinterpret_cast<int32_t*>(p) = (int32_t)node;
  const uint4 t = *reinterpret_cast<const uint4*>(local + (int64_t)r * nb + 8 * c);
  uint32_t* pw = reinterpret_cast<uint32_t*>(p + 4 + 8 * c);
  pw[0] = (t.x & 0xFFu) | ((t.x >> 16 & 0xFFu) << 8) | ((t.y & 0xFFu) << 16) |
          ((t.y >> 16 & 0xFFu) << 24);
  pw[1] = (t.z & 0xFFu) | ((t.z >> 16 & 0xFFu) << 8) | ((t.w & 0xFFu) << 16) |
          ((t.w >> 16 & 0xFFu) << 24);
  if (codes && node >= 0) *reinterpret_cast<uint4*>(codes + node * ldc + 8 * c) = t;
}

__device__ __forceinline__ unsigned long long wire_stamp(int64_t epoch, int64_t i) {
  return ((unsigned long long)epoch << 32) | (unsigned long long)(uint32_t)i;
}

__global__ void wire_winner_kernel(const uint8_t* __restrict__ recv, int64_t n, int rec,
                                   int64_t N, int64_t epoch,
                                   unsigned long long* __restrict__ winner) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int32_t node = *reinterpret_cast<const int32_t*>(recv + i * rec);
  if (node >= 0 && node < N) atomicMax(winner + node, wire_stamp(epoch, i));
}

__global__ void wire_scatter_kernel(const uint8_t* __restrict__ recv, int64_t n, int rec, int nb,
                                    int M, int64_t N, int64_t epoch,
                                    const unsigned long long* __restrict__ winner,
                                    int16_t* __restrict__ codes, int64_t ldc, int vec) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint8_t* p = recv + i * rec;
  const int32_t node = *reinterpret_cast<const int32_t*>(p);
  if (node < 0 || node >= N || winner[node] != wire_stamp(epoch, i)) return;
  int16_t* c = codes + (int64_t)node * ldc;
  if (vec) {
    const uint32_t* pw = reinterpret_cast<const uint32_t*>(p + 4);
    for (int b = 0; b < nb; b += 4) {
      const uint32_t w = pw[b / 4];
      *reinterpret_cast<uint2*>(c + b) =
          make_uint2((w & 0xFFu) | ((w >> 8 & 0xFFu) << 16), (w >> 16 & 0xFFu) | ((w >> 24) << 16));
    }
  } else if (wire_code_bytes(M) == 1) {
    for (int b = 0; b < nb; ++b) c[b] = (int16_t)p[4 + b];
  } else {
    const int16_t* q = reinterpret_cast<const int16_t*>(p + 4);
    for (int b = 0; b < nb; ++b) c[b] = q[b];
  }
}

// Thread (record, chunk of 8 codes): the table is read-only here, so the
// lanes of one record may sit in any wave or workgroup.
__global__ void wire_scatter8_kernel(const uint8_t* __restrict__ recv, int64_t n, int rec,
                                     int nb, int64_t N, int64_t epoch,
                                     const unsigned long long* __restrict__ winner,
                                     int16_t* __restrict__ codes, int64_t ldc) {
  const int ch = nb >> 3;
  const int64_t tix = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (tix >= n * ch) return;
  const int64_t i = tix / ch;
  const int c = (int)(tix % ch);
  const uint8_t* p = recv + i * rec;
  const int32_t node = *reinterpret_cast<const int32_t*>(p);
  if (node < 0 || node >= N || winner[node] != wire_stamp(epoch, i)) return;
  const uint32_t* pw = reinterpret_cast<const uint32_t*>(p + 4 + 8 * c);
  const uint32_t w0 = pw[0], w1 = pw[1];
  *reinterpret_cast<uint4*>(codes + (int64_t)node * ldc + 8 * c) =
      make_uint4((w0 & 0xFFu) | ((w0 >> 8 & 0xFFu) << 16), (w0 >> 16 & 0xFFu) | ((w0 >> 24) << 16),
                 (w1 & 0xFFu) | ((w1 >> 8 & 0xFFu) << 16), (w1 >> 16 & 0xFFu) | ((w1 >> 24) << 16));
}

}  // namespace vqgnn

using namespace vqgnn;

extern "C" int32_t vqgnn_codes_wire_record(int32_t nb, int32_t M) {
  return wire_record_bytes(nb, M);
}

extern "C" int vqgnn_pack_codes(const int64_t* batch_idx, int32_t B, const int16_t* local,
                                int32_t nb, int32_t M, int32_t max_B, uint8_t* send,
                                int16_t* codes, int64_t ldc, vqgnn_stream_t stream) {
  clear_error();
  VQGNN_REQUIRE(B >= 0 && max_B >= B && nb > 0 && M > 0 && M <= 32768,
                "pack_codes: bad shape (B=%d max_B=%d nb=%d M=%d)", B, max_B, nb, M);
  if (max_B == 0) return VQGNN_OK;
  VQGNN_REQUIRE(send && (B == 0 || (batch_idx && local)), "pack_codes: null pointer");
  // word-wise path: uint8 wire, 4 | nb, 8-byte aligned local rows and codes rows
  const int vec = M <= 256 && nb % 4 == 0 && ((uintptr_t)local & 7) == 0 &&
                  (!codes || (((uintptr_t)codes & 7) == 0 && ldc % 4 == 0));
  const bool vec8 = M <= 256 && nb % 8 == 0 && ((uintptr_t)local & 15) == 0 &&
                    (!codes || (((uintptr_t)codes & 15) == 0 && ldc % 8 == 0));
  if (vec8) {
    const int64_t nt = (int64_t)max_B * (nb / 8);
    hipLaunchKernelGGL(pack_codes8_kernel, dim3((unsigned)((nt + 255) / 256)), dim3(256), 0,
                       as_stream(stream), batch_idx, B, local, nb, max_B, send, codes, ldc);
  } else {
    hipLaunchKernelGGL(pack_codes_kernel, dim3((max_B + 255) / 256), dim3(256), 0,
                       as_stream(stream), batch_idx, B, local, nb, M, max_B, send, codes, ldc,
                       vec);
  }
  return check_launch("pack_codes");
}

extern "C" int vqgnn_scatter_wire(const uint8_t* recv, int64_t n_records, int32_t nb, int32_t M,
                                  int64_t* winner, int64_t epoch, int64_t N, int16_t* codes,
                                  int64_t ldc, vqgnn_stream_t stream) {
  clear_error();
  VQGNN_REQUIRE(n_records >= 0 && n_records < ((int64_t)1 << 32) && nb > 0 && M > 0 && N >= 0,
                "scatter_wire: bad shape");
  VQGNN_REQUIRE(epoch >= 1 && epoch < ((int64_t)1 << 31), "scatter_wire: epoch %lld outside [1, 2^31)",
                (long long)epoch);
  if (n_records == 0) return VQGNN_OK;
  VQGNN_REQUIRE(recv && winner && codes, "scatter_wire: null pointer");
  const int rec = wire_record_bytes(nb, M);
  unsigned long long* win = reinterpret_cast<unsigned long long*>(winner);
  const dim3 grid((unsigned)((n_records + 255) / 256));
  hipLaunchKernelGGL(wire_winner_kernel, grid, dim3(256), 0, as_stream(stream), recv, n_records,
                     rec, N, epoch, win);
  if (M <= 256 && nb % 8 == 0 && ((uintptr_t)codes & 15) == 0 && ldc % 8 == 0) {
    const int64_t nt = n_records * (nb / 8);
    hipLaunchKernelGGL(wire_scatter8_kernel, dim3((unsigned)((nt + 255) / 256)), dim3(256), 0,
                       as_stream(stream), recv, n_records, rec, nb, N, epoch, win, codes, ldc);
    return check_launch("scatter_wire");
  }
  const int vec = M <= 256 && nb % 4 == 0 && ((uintptr_t)codes & 7) == 0 && ldc % 4 == 0;
  hipLaunchKernelGGL(wire_scatter_kernel, grid, dim3(256), 0, as_stream(stream), recv, n_records,
                     rec, nb, M, N, epoch, win, codes, ldc, vec);
  return check_launch("scatter_wire");
}
