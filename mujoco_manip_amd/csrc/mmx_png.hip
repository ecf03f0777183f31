// Batched PNG encoder for gfx950 (LeRobot stores `dtype: image` features as
// embedded PNG frames, generate_dataset.py:250-260).  The camera images never leave the device
// raw: each RGB8 image becomes a complete PNG file in one workgroup, so the host receives
// compressed bytes (flat-shaded renders compress ~8x) and does no image work.
//
// One 256-lane workgroup per image (128 lanes for images of at most 128 rows):
//   1. rows in parallel (one row per lane): the PNG scanline (filter byte 0 + RGB bytes) is parsed
//      greedily into deflate symbols with two match candidates, the same pixel 3 bytes back and
//      the byte one scanline above (distance 3 S + 1); matches stay inside their row, so every
//      row parses independently.  One pass writes each row's bits (fixed Huffman codes, RFC 1951
//      §3.2.6) to a row-private scratch stream and counts them, with the row's Adler-32 partial
//      sums; a workgroup scan then gives every row its bit offset in the single final block;
//   2. every lane assembles whole dwords of the block from the rows that overlap them (no atomics),
//      then the zlib stream (header 78 01, block, Adler-32) is cut into IDAT chunks of kChunk
//      bytes written after the signature and IHDR; one lane per chunk computes its CRC-32; IEND
//      closes the file.  The size goes to sizes[image].
// Valid for any PNG decoder (a fixed-Huffman block, standard chunks); tests/test_png.py decodes
// with PIL and zlib and compares pixels exactly.
#include <hip/hip_runtime.h>
#include <stdint.h>

#define PNG_WG 256
static constexpr int kChunk = 512;  // IDAT data bytes per chunk (12 bytes of framing each)
static constexpr int kMaxMatch = 258;

__host__ __device__ inline int64_t png_row_words(int width) {  // row scratch: worst case 9 bits per byte
  return ((int64_t)(3 * width + 1) * 9 + 31) / 32 + 1;
}
__host__ __device__ inline int64_t png_zlib_bound(int width, int height) {
  const int64_t bits = 3 + (int64_t)height * (3 * width + 1) * 9 + 7;
  return 2 + (bits + 7) / 8 + 4;
}
// worst-case PNG size: signature + IHDR + chunked IDAT + IEND
__host__ __device__ inline int64_t png_bound(int width, int height) {
  const int64_t z = png_zlib_bound(width, height);
  return 8 + 25 + z + 12 * ((z + kChunk - 1) / kChunk) + 12;
}

__device__ inline uint32_t bit_reverse(uint32_t v, int n) { return __builtin_bitreverse32(v) >> (32 - n); }

// fixed-Huffman literal / length symbol -> (reversed code, bits)
__device__ inline void lit_code(int sym, uint32_t& code, int& nb) {
  if (sym < 144) { code = 0x30 + sym; nb = 8; }
  else if (sym < 256) { code = 0x190 + (sym - 144); nb = 9; }
  else if (sym < 280) { code = sym - 256; nb = 7; }
  else { code = 0xC0 + (sym - 280); nb = 8; }
  code = bit_reverse(code, nb);
}
// match length 3..258 -> symbol 257..285, extra bits, extra value
__device__ inline void len_sym(int len, int& sym, int& eb, int& ev) {
  if (len == 258) { sym = 285; eb = 0; ev = 0; return; }
  if (len <= 10) { sym = 254 + len; eb = 0; ev = 0; return; }
  // lengths 11..257: groups of 4 codes per extra-bit count e = 1..5, base 3 + 4 * 2^e
  const int v = len - 3;               // 8 .. 254
  const int e = 29 - __builtin_clz(v);  // floor(log2 v) - 2 (v >= 8 -> e >= 1)
  const int base = (4 + ((v >> e) - 4)) << e;  // (4 + q) << e with q = (v >> e) - 4 in 0..3
  sym = 265 + 4 * (e - 1) + ((v >> e) - 4);
  eb = e;
  ev = v - base;
}
// distance 1..32768 -> code 0..29, extra bits, extra value
__device__ inline void dist_code(int d, int& code, int& eb, int& ev) {
  if (d <= 4) { code = d - 1; eb = 0; ev = 0; return; }
  const int v = d - 1;
  const int e = 30 - __builtin_clz(v);  // floor(log2 v) - 1
  const int hi = (v >> e) & 1;
  code = 2 * e + 2 + hi;
  eb = e;
  ev = v - ((2 + hi) << e);
}

struct BitSink {  // LSB-first bit writer into a row-private word stream
  uint32_t* w;
  uint64_t acc;
  int n;
  int64_t words;
  __device__ void put(uint32_t v, int nb) {
    acc |= (uint64_t)v << n;
    n += nb;
    if (n >= 32) {
      w[words++] = (uint32_t)acc;
      acc >>= 32;
      n -= 32;
    }
  }
  __device__ void flush() {
    if (n > 0) w[words++] = (uint32_t)acc;
  }
};

// row r's scanline byte t (t = 0: filter byte 0, else RGB byte t - 1)
__device__ inline int scan_byte(const uint8_t* row, int t) { return t == 0 ? 0 : row[t - 1]; }

// length of the common prefix of a[0, lim) and b[0, lim): 4 bytes per step (one compare of two
// 4-byte loads, independent of each other), so a long match is a quarter of the dependent load
// round trips of a byte-at-a-time walk; reads stay inside [0, lim)
__device__ inline int run_len(const uint8_t* a, const uint8_t* b, int lim) {
  int m = 0;
  for (; m + 4 <= lim; m += 4) {
    uint32_t x, y;
    __builtin_memcpy(&x, a + m, 4);
    __builtin_memcpy(&y, b + m, 4);
    if (x != y) return m + (__builtin_ctz(x ^ y) >> 3);
  }
  while (m < lim && a[m] == b[m]) m++;
  return m;
}

// greedy parse of one scanline; EMIT = false counts bits, true writes them
template <bool EMIT>
__device__ int64_t parse_row(const uint8_t* row, const uint8_t* above, int L1, BitSink* bs) {
  int64_t bits = 0;
  const int dfar = L1;  // one scanline back
  int t = 0;
  while (t < L1) {
    const int lim = min(kMaxMatch, L1 - t);
    int m2 = 0, m1 = 0;
    if (above) {  // the byte above (filter bytes are both 0)
      m2 = t == 0 ? 1 + run_len(row, above, lim - 1) : run_len(row + t - 1, above + t - 1, lim);
    }
    if (t >= 4) {  // the same channel one pixel back (inside the row)
      m1 = run_len(row + t - 1, row + t - 4, lim);
    } else if (t == 3) {  // (its first byte is compared with the filter byte 0)
      m1 = row[2] == 0 ? 1 + run_len(row + 3, row, lim - 1) : 0;
    }
    const bool near = m1 >= m2;  // ties: the 3-byte distance (no extra bits)
    const int m = near ? m1 : m2;
    if (m >= 3) {
      int sym, eb, ev, dc, deb, dev;
      len_sym(m, sym, eb, ev);
      dist_code(near ? 3 : dfar, dc, deb, dev);
      uint32_t code;
      int nb;
      lit_code(sym, code, nb);
      bits += nb + eb + 5 + deb;
      if (EMIT) {
        bs->put(code, nb);
        if (eb) bs->put((uint32_t)ev, eb);
        bs->put(bit_reverse((uint32_t)dc, 5), 5);
        if (deb) bs->put((uint32_t)dev, deb);
      }
      t += m;
    } else {
      uint32_t code;
      int nb;
      lit_code(scan_byte(row, t), code, nb);
      bits += nb;
      if (EMIT) bs->put(code, nb);
      t++;
    }
  }
  return bits;
}

// zlib byte j inside the chunked IDAT area: chunk j / kChunk, after its 8-byte length + type
__device__ inline int64_t zpos(int64_t j) { return j + 12 * (j / kChunk) + 8; }

__device__ inline void put_be32(uint8_t* p, uint32_t v) {
  p[0] = (uint8_t)(v >> 24); p[1] = (uint8_t)(v >> 16); p[2] = (uint8_t)(v >> 8); p[3] = (uint8_t)v;
}

__device__ uint32_t crc_table(int k) {  // CRC-32 (IEEE, reflected) table entry, computed on the fly
  uint32_t c = (uint32_t)k;
  for (int j = 0; j < 8; j++) c = (c & 1u) ? 0xEDB88320u ^ (c >> 1) : (c >> 1);
  return c;
}

// WG lanes per image: one row per lane, so an image of at most 128 rows runs on 128 lanes (no idle
// waves holding the CU's wave slots during the row parses, which are serial per lane: the encoder's
// speed is the number of rows in flight per CU)
template <int WG>
__device__ void png_encode(const uint8_t* rgb, int64_t img_stride, int W, int H, uint8_t* out, int64_t out_stride,
                           int32_t* sizes, uint32_t* scratch) {
  __shared__ int32_t s_off[1025];  // bit offset of each row in the block (H <= 1024, W <= 10922: < 2^29)
  __shared__ uint64_t s_a1[WG], s_a2[WG];
  __shared__ uint32_t s_crc[256];
  __shared__ int64_t s_tot;
  const int img = blockIdx.x, tid = threadIdx.x;
  const uint8_t* im = rgb + (int64_t)img * img_stride;
  const int L = 3 * W, L1 = L + 1;
  const int64_t rw = png_row_words(W);
  uint32_t* scr = scratch + (int64_t)img * H * rw;
  uint8_t* o = out + (int64_t)img * out_stride;
  for (int k = tid; k < 256; k += WG) s_crc[k] = crc_table(k);
  // one pass: each row's bits into its private stream, its bit count, and the Adler-32 partial sums
  // (s1: sum of bytes, s2: sum of (n - i) byte_i)
  const uint64_t n = (uint64_t)H * L1;
  uint64_t a1 = 0, a2 = 0;
  for (int r = tid; r < H; r += WG) {
    const uint8_t* row = im + (int64_t)r * L;
    BitSink bs{scr + (int64_t)r * rw, 0ull, 0, 0};  // (the row's stream is private: no offset needed yet)
    s_off[r + 1] = (int32_t)parse_row<true>(row, r ? row - L : nullptr, L1, &bs);
    bs.flush();
    const uint64_t i0 = (uint64_t)r * L1 + 1;  // the filter byte (0) adds nothing
    for (int k = 0; k < L; k++) {
      const uint64_t b = row[k];
      a1 += b;
      a2 += (n - (i0 + k)) * b;
    }
  }
  s_a1[tid] = a1;
  s_a2[tid] = a2;
  __syncthreads();
  if (tid == 0) {  // exclusive scan of the row bit counts after the 3 block-header bits; Adler-32
    s_off[0] = 3;
    for (int r = 0; r < H; r++) s_off[r + 1] += s_off[r];
    uint64_t A1 = 1, A2 = n;  // s2 = n (the initial 1 of s1 counted at each byte) + sum (n - i) b_i
    for (int k = 0; k < WG; k++) {
      A1 += s_a1[k];
      A2 += s_a2[k];
    }
    s_a1[0] = ((A2 % 65521u) << 16) | (A1 % 65521u);
    s_tot = s_off[H] + 7;  // + end of block (code 256: seven 0 bits)
  }
  __syncthreads();
  __threadfence();  // the streams are read by other lanes of the workgroup
  __syncthreads();
  const uint32_t adler = (uint32_t)s_a1[0];
  const int64_t nbits = s_tot, nd = (nbits + 7) / 8;  // deflate bytes
  const int64_t zlen = 2 + nd + 4;
  const int64_t nchunk = (zlen + kChunk - 1) / kChunk;
  uint8_t* idat = o + 8 + 25;
  // deflate block dword w: the header bits and the rows overlapping [32 w, 32 w + 32); written as
  // bytes into the chunked layout (zlib byte j lives at idat + zpos(j))
  const int64_t nw = (nbits + 31) / 32;
  for (int64_t w = tid; w < nw; w += WG) {
    const int64_t b0 = 32 * w, b1 = b0 + 32;
    uint32_t v = w == 0 ? 3u : 0u;  // BFINAL = 1, BTYPE = 01 (fixed Huffman)
    int lo = 0, hi = H;             // first row whose range ends after b0
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (s_off[mid + 1] <= b0) lo = mid + 1;
      else hi = mid;
    }
    for (int r = lo; r < H && s_off[r] < b1; r++) {
      const int64_t rs = s_off[r], re = s_off[r + 1];
      const int64_t lb = max(b0, rs) - rs;  // local bit in the row's stream
      const int64_t take = min(b1, re) - (rs + lb);
      if (take <= 0) continue;
      const uint32_t* rwp = scr + (int64_t)r * rw;
      const int64_t k = lb >> 5;
      const int s = (int)(lb & 31);
      uint64_t bits = rwp[k];
      if (s + take > 32) bits |= (uint64_t)rwp[k + 1] << 32;
      bits >>= s;
      if (take < 32) bits &= (1ull << take) - 1;
      v |= (uint32_t)(bits << (rs + lb - b0));
    }
    for (int q = 0; q < 4; q++) {
      const int64_t j = 2 + 4 * w + q;  // zlib byte
      if (j - 2 < nd) idat[zpos(j)] = (uint8_t)(v >> (8 * q));
    }
  }
  if (tid == 0) {  // signature, IHDR, zlib header and Adler-32, chunk headers, IEND, size
    const uint8_t sig[8] = {0x89, 'P', 'N', 'G', 0x0D, 0x0A, 0x1A, 0x0A};
    for (int k = 0; k < 8; k++) o[k] = sig[k];
    uint8_t* ih = o + 8;
    put_be32(ih, 13);
    ih[4] = 'I'; ih[5] = 'H'; ih[6] = 'D'; ih[7] = 'R';
    put_be32(ih + 8, (uint32_t)W);
    put_be32(ih + 12, (uint32_t)H);
    ih[16] = 8; ih[17] = 2; ih[18] = 0; ih[19] = 0; ih[20] = 0;  // 8-bit RGB, deflate, no interlace
    uint32_t c = 0xFFFFFFFFu;
    for (int k = 4; k < 21; k++) c = crc_table((c ^ ih[k]) & 255) ^ (c >> 8);
    put_be32(ih + 21, ~c);
    const uint8_t zh[2] = {0x78, 0x01};
    for (int j = 0; j < 2; j++) idat[zpos(j)] = zh[j];
    for (int q = 0; q < 4; q++) {
      const int64_t j = 2 + nd + q;
      idat[zpos(j)] = (uint8_t)(adler >> (24 - 8 * q));
    }
    for (int64_t ch = 0; ch < nchunk; ch++) {
      uint8_t* hp = idat + ch * (kChunk + 12);
      put_be32(hp, (uint32_t)min((int64_t)kChunk, zlen - ch * kChunk));
      hp[4] = 'I'; hp[5] = 'D'; hp[6] = 'A'; hp[7] = 'T';
    }
    uint8_t* ie = idat + nchunk * 12 + zlen;
    const uint8_t iend[12] = {0, 0, 0, 0, 'I', 'E', 'N', 'D', 0xAE, 0x42, 0x60, 0x82};
    for (int k = 0; k < 12; k++) ie[k] = iend[k];
    sizes[img] = (int32_t)(8 + 25 + nchunk * 12 + zlen + 12);
  }
  __threadfence();
  __syncthreads();
  for (int64_t ch = tid; ch < nchunk; ch += WG) {  // one lane per chunk: CRC of type + data
    uint8_t* hp = idat + ch * (kChunk + 12);
    const int64_t len = min((int64_t)kChunk, zlen - ch * kChunk);
    uint32_t c = 0xFFFFFFFFu;
    for (int64_t k = 4; k < 8 + len; k++) c = s_crc[(c ^ hp[k]) & 255] ^ (c >> 8);
    put_be32(hp + 8 + len, ~c);
  }
}

extern "C" __global__ void __launch_bounds__(PNG_WG)
mmx_png_kernel(const uint8_t* rgb, int64_t img_stride, int W, int H, uint8_t* out, int64_t out_stride,
               int32_t* sizes, uint32_t* scratch) {
  png_encode<PNG_WG>(rgb, img_stride, W, H, out, out_stride, sizes, scratch);
}
extern "C" __global__ void __launch_bounds__(128)
mmx_png_kernel_128(const uint8_t* rgb, int64_t img_stride, int W, int H, uint8_t* out, int64_t out_stride,
                   int32_t* sizes, uint32_t* scratch) {
  png_encode<128>(rgb, img_stride, W, H, out, out_stride, sizes, scratch);
}

// packed[offsets[i] ..] = the first sizes[i] bytes of image i's slot
extern "C" __global__ void __launch_bounds__(PNG_WG)
mmx_png_pack_kernel(const uint8_t* out, int64_t out_stride, const int32_t* sizes, const int64_t* offsets, uint8_t* packed) {
  const int i = blockIdx.x;
  const uint8_t* src = out + (int64_t)i * out_stride;
  uint8_t* dst = packed + offsets[i];
  for (int k = threadIdx.x; k < sizes[i]; k += PNG_WG) dst[k] = src[k];
}

extern "C" int64_t mmx_png_bound_bytes(int width, int height) { return png_bound(width, height); }
extern "C" int64_t mmx_png_scratch_bytes(int width, int height) { return (int64_t)height * png_row_words(width) * 4; }

extern "C" hipError_t mmx_launch_png(const uint8_t* rgb, int64_t img_stride, int n, int W, int H, uint8_t* out,
                                     int64_t out_stride, int32_t* sizes, uint32_t* scratch, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  if (W <= 0 || H <= 0 || H > 1024 || out_stride < png_bound(W, H)) return hipErrorInvalidValue;
  if (H <= 128)
    hipLaunchKernelGGL(mmx_png_kernel_128, dim3(n), dim3(128), 0, st, rgb, img_stride, W, H, out, out_stride, sizes,
                       scratch);
  else
    hipLaunchKernelGGL(mmx_png_kernel, dim3(n), dim3(PNG_WG), 0, st, rgb, img_stride, W, H, out, out_stride, sizes,
                       scratch);
  return hipGetLastError();
}
extern "C" hipError_t mmx_launch_png_pack(const uint8_t* out, int64_t out_stride, const int32_t* sizes,
                                          const int64_t* offsets, int n, uint8_t* packed, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(mmx_png_pack_kernel, dim3(n), dim3(PNG_WG), 0, st, out, out_stride, sizes, offsets, packed);
  return hipGetLastError();
}

// ============================================================================ image statistics
// Per-image, per-channel min / max / sum / sum of squares of RGB8 images (LeRobot's image feature
// statistics, generate_dataset.py:250-260; the dataset scales them to [0, 1]): out[i] = int64
// [min R G B, max R G B, sum R G B, sumsq R G B], exact integers.  One 256-lane workgroup per image,
// a single pass over its bytes (HBM-bound: one read of the frames the PNG encoder reads anyway),
// replacing the dataset's torch reductions (4-6 passes with int32 / int64 widening copies).
// Fast path (image base 4-byte aligned, pixel count a multiple of 4): a lane reads 3 dwords = 4
// pixels; the channels' bytes of the 3 dwords fall on disjoint byte lanes, so each channel's 4
// bytes are gathered into one dword with AND / OR, then v_dot4_u32_u8 against 0x01010101 (sum)
// and against itself (sum of squares).  Otherwise one pixel per step.
#define IST_WG 256
__device__ __forceinline__ void ist_minmax4(uint32_t x, uint32_t& mn, uint32_t& mx) {
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const uint32_t b = (x >> (8 * k)) & 255u;
    mn = min(mn, b);
    mx = max(mx, b);
  }
}
__device__ __forceinline__ uint64_t ist_wave_sum(uint64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ uint32_t ist_wave_min(uint32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = min(v, (uint32_t)__shfl_xor((int)v, o, 64));
  return v;
}
__device__ __forceinline__ uint32_t ist_wave_max(uint32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, o, 64));
  return v;
}
extern "C" __global__ void __launch_bounds__(IST_WG)
mmx_image_stats_kernel(const uint8_t* rgb, int64_t img_stride, int64_t npx, int64_t* out) {
  const int img = blockIdx.x, tid = threadIdx.x;
  const uint8_t* im = rgb + (int64_t)img * img_stride;
  uint32_t mn[3] = {255u, 255u, 255u}, mx[3] = {0u, 0u, 0u};
  uint64_t sm[3] = {0, 0, 0}, sq[3] = {0, 0, 0};
  if ((reinterpret_cast<uintptr_t>(im) & 3) == 0 && (npx & 3) == 0) {
    const uint32_t* w = reinterpret_cast<const uint32_t*>(im);
    const int64_t ng = npx >> 2;  // groups of 4 pixels = 3 dwords
    // (per-lane 32-bit partial sums: at most 4 x 255^2 per group and npx / 4 / 256 groups per lane
    // before the 64-bit fold below, i.e. safe for images up to 4096 x 4096)
    uint32_t s32[3] = {0u, 0u, 0u}, q32[3] = {0u, 0u, 0u};
    for (int64_t g = tid; g < ng; g += IST_WG) {
      const uint32_t w0 = w[3 * g], w1 = w[3 * g + 1], w2 = w[3 * g + 2];
      // bytes: w0 = R0 G0 B0 R1, w1 = G1 B1 R2 G2, w2 = B2 R3 G3 B3 (little-endian byte order)
      const uint32_t xr = (w0 & 0xFF0000FFu) | (w1 & 0x00FF0000u) | (w2 & 0x0000FF00u);
      const uint32_t xg = (w0 & 0x0000FF00u) | (w1 & 0xFF0000FFu) | (w2 & 0x00FF0000u);
      const uint32_t xb = (w0 & 0x00FF0000u) | (w1 & 0x0000FF00u) | (w2 & 0xFF0000FFu);
      const uint32_t xc[3] = {xr, xg, xb};
#pragma unroll
      for (int c = 0; c < 3; c++) {
        s32[c] = __builtin_amdgcn_udot4(xc[c], 0x01010101u, s32[c], false);
        q32[c] = __builtin_amdgcn_udot4(xc[c], xc[c], q32[c], false);
        ist_minmax4(xc[c], mn[c], mx[c]);
      }
    }
#pragma unroll
    for (int c = 0; c < 3; c++) {
      sm[c] = s32[c];
      sq[c] = q32[c];
    }
  } else {
    for (int64_t p = tid; p < npx; p += IST_WG) {
#pragma unroll
      for (int c = 0; c < 3; c++) {
        const uint32_t b = im[3 * p + c];
        mn[c] = min(mn[c], b);
        mx[c] = max(mx[c], b);
        sm[c] += b;
        sq[c] += b * b;
      }
    }
  }
  __shared__ uint64_t red[IST_WG / 64][12];
  const int wv = tid >> 6;
#pragma unroll
  for (int c = 0; c < 3; c++) {
    const uint32_t a = ist_wave_min(mn[c]), b = ist_wave_max(mx[c]);
    const uint64_t s1 = ist_wave_sum(sm[c]), s2 = ist_wave_sum(sq[c]);
    if ((tid & 63) == 0) {
      red[wv][c] = a;
      red[wv][3 + c] = b;
      red[wv][6 + c] = s1;
      red[wv][9 + c] = s2;
    }
  }
  __syncthreads();
  if (tid < 12) {
    uint64_t v = red[0][tid];
    for (int k = 1; k < IST_WG / 64; k++) {
      const uint64_t u = red[k][tid];
      v = tid < 3 ? min(v, u) : (tid < 6 ? max(v, u) : v + u);
    }
    out[(int64_t)img * 12 + tid] = (int64_t)v;
  }
}
extern "C" hipError_t mmx_launch_image_stats(const uint8_t* rgb, int64_t img_stride, int n, int64_t npx, int64_t* out,
                                             hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(mmx_image_stats_kernel, dim3(n), dim3(IST_WG), 0, st, rgb, img_stride, npx, out);
  return hipGetLastError();
}
