// Whisper front end on gfx950: log-mel spectrogram and the per-video-frame
// audio feature gather.
//
//  * log_mel_kernel: whisper/audio.py:92-125 (torch.stft n_fft 400, hop 160,
//    periodic Hann, centre reflect padding, last frame dropped; |X|^2; 80-band
//    filterbank; log10(max(., 1e-10))).  One block owns MEL_FR consecutive frames:
//    windowed samples + a 400-entry twiddle table live in LDS, the 201-bin power
//    spectrum goes to LDS, then each thread forms mel bands.  The DFT is direct
//    (400 x 201 fp32 MACs per frame, ~0.5 GFLOP per 30 s) -- VALU work that
//    finishes in microseconds; it stays fp32 like the reference.  Every block
//    folds its maximum into one ordered-uint slot for the clip-global
//    `max - 8` floor.
//  * mel_norm_kernel: floor + (x + 4) / 4, written frame-major bf16 [T_pad][80]
//    (the NHWC input of conv1), zero past T (pad_or_trim after normalisation,
//    whisper/transcribe.py segment loop).
//  * audio_chunks_kernel: Audio2Feature.get_sliced_feature / feature2chunks
//    (audio2feature.py:24-49, 85-100): chunk i row j = feature[clamp(c-2L+j/layers)]
//    [layer j%layers], c = int(i * 50 / fps) evaluated in double like Python.
#include "ls_common.h"

namespace ls {

constexpr int N_FFT = 400, HOP = 160, N_FREQ = N_FFT / 2 + 1, MEL_FR = 8;

__device__ __forceinline__ unsigned ord_enc(float v) {
  const unsigned b = __float_as_uint(v);
  return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}
__device__ __forceinline__ float ord_dec(unsigned u) {
  return __uint_as_float((u & 0x80000000u) ? (u & 0x7fffffffu) : ~u);
}

__global__ void __launch_bounds__(256)
log_mel_kernel(const float* __restrict__ audio, long n_samples, int T, const float* __restrict__ filters, int n_mels,
               float* __restrict__ logmel, unsigned* __restrict__ gmax) {
  __shared__ float xw[MEL_FR][N_FFT];
  __shared__ float cs[N_FFT], sn[N_FFT];
  __shared__ float pw[MEL_FR][N_FREQ + 3];
  __shared__ float wmax[4];
  const int tid = threadIdx.x;
  const int t0 = blockIdx.x * MEL_FR;
  for (int i = tid; i < N_FFT; i += 256) {
    float s, c;
    sincospif(2.0f * (float)i / (float)N_FFT, &s, &c);
    cs[i] = c;
    sn[i] = s;
  }
  __syncthreads();
  for (int i = tid; i < MEL_FR * N_FFT; i += 256) {
    const int f = i / N_FFT, n = i - f * N_FFT;
    const int t = t0 + f;
    float v = 0.f;
    if (t < T) {
      long j = (long)t * HOP + n - N_FFT / 2;  // centre padding, reflect
      if (j < 0) j = -j;
      if (j >= n_samples) j = 2 * (n_samples - 1) - j;
      const float hann = 0.5f - 0.5f * cs[n];  // periodic Hann
      v = audio[j] * hann;
    }
    xw[f][n] = v;
  }
  __syncthreads();
  for (int p = tid; p < MEL_FR * N_FREQ; p += 256) {
    const int f = p / N_FREQ, k = p - f * N_FREQ;
    float re = 0.f, im = 0.f;
    int idx = 0;
    const float* x = xw[f];
#pragma unroll 8
    for (int n = 0; n < N_FFT; ++n) {
      re += x[n] * cs[idx];
      im -= x[n] * sn[idx];
      idx += k;
      if (idx >= N_FFT) idx -= N_FFT;
    }
    pw[f][k] = re * re + im * im;
  }
  __syncthreads();
  float m = -INFINITY;
  for (int p = tid; p < MEL_FR * n_mels; p += 256) {
    const int f = p / n_mels, b = p - f * n_mels;
    const int t = t0 + f;
    if (t >= T) continue;
    const float* fr = filters + (long)b * N_FREQ;
    float s = 0.f;
    for (int k = 0; k < N_FREQ; ++k) s += fr[k] * pw[f][k];
    const float l = log10f(fmaxf(s, 1e-10f));
    logmel[(long)t * n_mels + b] = l;
    m = fmaxf(m, l);
  }
  m = wave_max(m);
  if ((tid & 63) == 0) wmax[tid >> 6] = m;
  __syncthreads();
  if (tid == 0) {
    const float bm = fmaxf(fmaxf(wmax[0], wmax[1]), fmaxf(wmax[2], wmax[3]));
    if (bm > -INFINITY) atomicMax(gmax, ord_enc(bm));
  }
}

__global__ void mel_norm_kernel(const float* __restrict__ logmel, int T, int n_mels, long T_pad,
                                const unsigned* __restrict__ gmax, u16* __restrict__ out) {
  const float floor_v = ord_dec(*gmax) - 8.0f;
  const long n = T_pad * n_mels;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const long t = i / n_mels;
    float v = 0.f;
    if (t < T) v = (fmaxf(logmel[i], floor_v) + 4.0f) / 4.0f;
    out[i] = f2bf(v);
  }
}

__global__ void audio_chunks_kernel(const u16* __restrict__ feat, long ld_row, int T, int layers, int C, int n_chunks,
                                    double fps, int left, int right, void* __restrict__ out, int out_f32) {
  const int rows = (left + right + 1) * 2 * layers;  // 50 for [2, 2] and 5 layers
  const int CC = C / 8;
  const long n = (long)n_chunks * rows * CC;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const int cc = (int)(i % CC);
    const long r = i / CC;
    const int j = (int)(r % rows);
    const int ch = (int)(r / rows);
    const int center = (int)((double)ch * 50.0 / fps);  // int(vid_idx * 50 / fps)
    int idx = center - left * 2 + j / layers;
    idx = idx < 0 ? 0 : (idx > T - 1 ? T - 1 : idx);
    const uint4 v = *(const uint4*)(feat + (long)idx * ld_row + (long)(j % layers) * C + cc * 8);
    if (out_f32) {
      float f[8];
      unpack8(v, f);
      float* o = (float*)out + r * C + cc * 8;
      *(float4*)o = make_float4(f[0], f[1], f[2], f[3]);
      *(float4*)(o + 4) = make_float4(f[4], f[5], f[6], f[7]);
    } else {
      *(uint4*)((u16*)out + r * C + cc * 8) = v;
    }
  }
}

}  // namespace ls

using namespace ls;

extern "C" size_t ls_log_mel_workspace_bytes(int64_t n_samples, int32_t n_mels) {
  const long T = n_samples / HOP;
  return 256 + (size_t)T * n_mels * sizeof(float);
}

extern "C" int ls_log_mel(const float* audio, int64_t n_samples, const float* filters, int32_t n_mels, int64_t t_pad,
                          uint16_t* out, void* workspace, size_t workspace_bytes, void* stream) {
  if (!audio || !filters || !out || n_samples < N_FFT / 2 + 1 || n_mels <= 0 || n_mels > 128)
    return fail(LS_ERR_INVALID, "ls_log_mel: bad arguments (need > 200 samples, n_mels <= 128)");
  const long T = n_samples / HOP;
  if (t_pad < T) return fail(LS_ERR_INVALID, "ls_log_mel: t_pad < number of frames");
  if (!workspace || workspace_bytes < ls_log_mel_workspace_bytes(n_samples, n_mels))
    return fail(LS_ERR_WORKSPACE, "ls_log_mel: workspace too small");
  hipStream_t s = (hipStream_t)stream;
  unsigned* gmax = (unsigned*)workspace;
  float* logmel = (float*)((char*)workspace + 256);
  if (hipMemsetAsync(gmax, 0, sizeof(unsigned), s) != hipSuccess) return fail(LS_ERR_LAUNCH, "ls_log_mel: memset");
  log_mel_kernel<<<(int)cdiv(T, MEL_FR), 256, 0, s>>>(audio, n_samples, (int)T, filters, n_mels, logmel, gmax);
  if (int rc = check_launch("log_mel_kernel")) return rc;
  const long n = t_pad * n_mels;
  mel_norm_kernel<<<(int)std::min<long>(cdiv(n, 256), 4096), 256, 0, s>>>(logmel, (int)T, n_mels, t_pad, gmax, out);
  return check_launch("mel_norm_kernel");
}

extern "C" int ls_audio_chunks(const uint16_t* feat, int64_t ld_row, int32_t T, int32_t layers, int32_t C,
                               int32_t n_chunks, double fps, int32_t left, int32_t right, void* out, int32_t out_f32,
                               void* stream) {
  if (!feat || !out || T <= 0 || layers <= 0 || C % 8 || ld_row % 8 || n_chunks < 0 || !(fps > 0) || left < 0 ||
      right < 0)
    return fail(LS_ERR_INVALID, "ls_audio_chunks: bad arguments");
  if (n_chunks == 0) return LS_OK;
  const long n = (long)n_chunks * (left + right + 1) * 2 * layers * (C / 8);
  audio_chunks_kernel<<<(int)std::min<long>(cdiv(n, 256), 8192), 256, 0, (hipStream_t)stream>>>(
      feat, ld_row, T, layers, C, n_chunks, fps, left, right, out, out_f32);
  return check_launch("audio_chunks_kernel");
}
