/*
 * aa.h -- C ABI of libaa.so, the MI355X (gfx950) hot path of the
 * audio-analysis window classifier.
 *
 * Every entry point is plain C: device pointers, sizes, an opaque handle and a
 * hipStream_t passed as void*.  No torch types cross this boundary.  Buffers
 * are owned by the caller (the Python host keeps them in torch-ROCm tensors);
 * the library allocates only per-handle constants (filterbank, twiddles,
 * packed weights) at create time, never inside a *_run / *_forward call, so
 * those calls can be captured into a HIP graph.
 *
 * Reference interfaces each group replaces (file:line in
 * TheCacophonyProject/audio-analysis, mounted at /root/reference):
 *   aa_fe_*      get_spect(...)                     src/identify_tracks.py:212-288
 *                  + normalize_data                 src/identify_tracks.py:202-209
 *                  + the per-window loop body       src/identify_tracks.py:163-193
 *                  + custommel.mel_spec / mel_f     src/custommel.py:19-63
 *   aa_model_*   load_model(path, meta)             src/identify_tracks.py:302-327
 *                model.predict(np.array(d))         src/identify_tracks.py:544
 *                MagTransform.call                  src/magtransformv2.py:19-21
 *   aa_track_mean  np.mean over models, windows     src/identify_tracks.py:547-551
 *   aa_span_nonzero  get_end                        src/identify_tracks.py:387-413
 *   aa_pcm_s16_to_f32  load_recording's s16 -> f32  src/identify_tracks.py:49-62
 *   aa_resample_poly   load_recording's resample     src/identify_tracks.py:49-62
 *   aa_sn_*      signal_noise                       src/identify_tracks.py:650-706
 *   aa_flac_*    load_recording's ffmpeg decode     src/identify_tracks.py:49-62
 *                  (FLAC; host memory, no GPU)
 *   aa_vorbis_*  load_recording's ffmpeg decode     src/identify_tracks.py:49-62
 *                  (Ogg Vorbis; host memory, no GPU)
 *
 * Return values: AA_OK (0) or an aa_status code; aa_last_error() gives a
 * thread-local message for the last failing call on this thread.
 */
#ifndef AA_H
#define AA_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define AA_ABI_VERSION 2

typedef enum aa_status {
    AA_OK = 0,
    AA_ERR_INVALID = 1,      /* bad argument / shape */
    AA_ERR_HIP = 2,          /* HIP runtime error */
    AA_ERR_UNSUPPORTED = 3,  /* layer pattern or size this build has no kernel for */
    AA_ERR_WORKSPACE = 4,    /* workspace too small */
} aa_status;

/* One analysis window of `win_len` samples, as a view into the recording:
 * samples [src, src + n_valid) of the PCM buffer, placed at offset pad_left
 * inside the window; every other window sample is 0 (np.pad,
 * src/identify_tracks.py:165-168).  16 bytes, device-resident array. */
typedef struct aa_window {
    int64_t src;
    int32_t n_valid;
    int32_t pad_left;
} aa_window;

/* Front-end configuration (the reference's metadata.txt keys,
 * src/identify_tracks.py:466-497). */
typedef struct aa_fe_config {
    int32_t win_len;   /* samples per window: int(sr * segment_length) */
    int32_t n_fft;     /* power of two, 1024..8192 */
    int32_t hop;       /* hop_length */
    int32_t n_mels;    /* rows of the filterbank */
    int32_t normalize; /* normalize_data before the STFT */
    int32_t db_scale;  /* librosa.power_to_db(ref=np.max) */
    float power;       /* |S| ** power before the filterbank */
    float amin;        /* power_to_db amin (1e-10) */
    float top_db;      /* power_to_db top_db (80) */
    int32_t mean_sub;  /* subtract each band's mean over time */
    int32_t channels;  /* repeat the single channel this many times */
    int32_t out_f16;   /* 1: aa_fe_run writes float16 log-mel (BASELINE configs[4]),
                        * 0: float32 (what get_spect returns) */
} aa_fe_config;

/* Per-window status flags written by aa_fe_run (device int32 array). */
#define AA_WIN_OK 0
#define AA_WIN_NONFINITE 1 /* librosa.util.valid_audio would raise */

int aa_abi_version(void);
const char* aa_last_error(void);

/* ---------------- front end: PCM windows -> log-mel ---------------- */
/* melfb: host float32 [n_mels][n_fft/2 + 1] dense filterbank (custommel.mel_f
 * or the Slaney filterbank); stored on the device in CSR form. */
int aa_fe_create(const aa_fe_config* cfg, const float* melfb, void** plan);
int aa_fe_destroy(void* plan);
/* frames per window T = 1 + win_len / hop */
int aa_fe_n_frames(const void* plan);
size_t aa_fe_workspace_bytes(const void* plan, int32_t max_windows);
/* out: device [n_win][n_mels][T][channels] (NHWC, H = mel band, W = frame),
 * the tensor get_spect returns per window: float32, or float16 (round to
 * nearest) when cfg.out_f16.
 * win_status: device int32 [n_win] (AA_WIN_*), may be NULL. */
int aa_fe_run(void* plan, const float* pcm, int64_t pcm_len, const aa_window* windows,
              int32_t n_win, void* out, int32_t* win_status, void* workspace,
              size_t workspace_bytes, void* stream);
/* Launch stages of aa_fe_run (0 fe_stats, 1 fe_stft_mel, 2 fe_db) and their
 * timing, same contract as aa_model_stage_* below. */
int aa_fe_n_stages(const void* plan);
int aa_fe_stage_info(const void* plan, int32_t stage, char* name, int32_t name_len,
                     double* flops_per_item, double* bytes_per_item);
int aa_fe_set_timing(void* plan, uint32_t stage_mask);
int aa_fe_stage_time(void* plan, int32_t stage, double* total_ms, int64_t* count);

/* ---------------- CNN: log-mel windows -> logits / probabilities ---------------- */
/* Supported layer sequences: [MagTransform] then Conv2D blocks (Conv2D
 * [BatchNormalization] [LeakyReLU|ReLU] [MaxPooling2D]) ending in either a
 * 1x1 Conv2D + GlobalMaxPool2D [+ sigmoid] head or GlobalMaxPool2D [+ Dense]
 * [+ sigmoid].  Tuned matrix-core kernels serve the build's model family
 * (stage names "conv_*"); any other conv shape or pool window runs a generic
 * f32 kernel (stage name "conv_generic_*"; not in the fp8 mode). */
typedef enum aa_op {
    AA_OP_CONV2D = 1,       /* Keras Conv2D, padding="valid", stride 1 */
    AA_OP_BATCHNORM = 2,    /* inference BatchNormalization (moving stats) */
    AA_OP_LEAKYRELU = 3,
    AA_OP_MAXPOOL2D = 4,    /* pool = strides, padding="valid" */
    AA_OP_GLOBALMAXPOOL2D = 5,
    AA_OP_SIGMOID = 6,
    AA_OP_MAGTRANSFORM = 7, /* x ** sigmoid(a) */
    AA_OP_RELU = 8,
    AA_OP_DENSE = 9,        /* after GlobalMaxPool2D: filters = units,
                             * off[0] = kernel [C_in][units], off[1] = bias */
} aa_op;

typedef struct aa_layer {
    int32_t op;      /* aa_op */
    int32_t kh, kw;  /* conv kernel or pool size */
    int32_t filters; /* conv output channels */
    float alpha;     /* leaky slope */
    float eps;       /* batchnorm epsilon */
    /* offsets (in floats) into the weight blob, -1 when absent:
     * conv: [0]=kernel (HWIO [kh][kw][cin][cout]), [1]=bias
     * batchnorm: [0]=gamma [1]=beta [2]=moving_mean [3]=moving_variance
     * magtransform: [0]=a */
    int64_t off[4];
} aa_layer;

typedef enum aa_precision {
    AA_PREC_F32 = 0,  /* f32 MFMA (exact f32 fma chain): the parity mode */
    AA_PREC_BF16 = 1, /* bf16 activations/weights, f32 accumulation */
    AA_PREC_FP8 = 2,  /* OCP e4m3fn activations/weights (per-output-channel weight
                       * scales), f32 accumulation; f32 log-mel input, the first
                       * conv on bf16 hi+lo as in AA_PREC_BF16 */
    AA_PREC_BF16X3 = 3, /* split bf16: f32 activations, operands split into
                         * bf16 hi + lo, hi*hi + hi*lo + lo*hi on bf16 MFMA
                         * with f32 accumulation (~17-bit products): meets the
                         * 1e-3 logit gate; the default of classify() */
} aa_precision;

int aa_model_create(const aa_layer* layers, int32_t n_layers, const float* blob, int64_t blob_len,
                    int32_t in_h, int32_t in_w, int32_t in_c, int32_t precision, void** model);
int aa_model_destroy(void* model);
int aa_model_n_outputs(const void* model);
size_t aa_model_workspace_bytes(const void* model, int32_t max_batch);
/* x: device [n][in_h][in_w][in_c], float32 (or float16 after
 * aa_model_set_input_f16(model, 1)); logits: device float32 [n][L]
 * (global-max outputs before the sigmoid); probs: [n][L] or NULL. */
int aa_model_forward(void* model, const void* x, int32_t n, float* logits, float* probs,
                     void* workspace, size_t workspace_bytes, void* stream);
/* Model input as float16 (aa_fe_config.out_f16): served when the first
 * conv is fused into the second (the build's model family: 3x3 C_in = 1 ->
 * 32 before a pooled 3x3/32 conv), which converts the log-mel to f32 as it
 * stages it; AA_ERR_UNSUPPORTED otherwise. */
int aa_model_set_input_f16(void* model, int32_t f16);

/* Per-stage timing of aa_model_forward (HIP events around each stage whose
 * bit is set in stage_mask, on the launch stream; 0 disables).  Used by
 * bench.py for the roofline of the dominant kernel.  stage_info reports the
 * algorithmic flops / HBM bytes of one window (item) through the stage. */
int aa_model_n_stages(const void* model);
int aa_model_stage_info(const void* model, int32_t stage, char* name, int32_t name_len,
                        double* flops_per_item, double* bytes_per_item);
int aa_model_set_timing(void* model, uint32_t stage_mask);
int aa_model_stage_time(void* model, int32_t stage, double* total_ms, int64_t* count);

/* ---------------- CNN graphs (DAG models: residual / squeeze-excite / depthwise) ---------------- */
/* Models that are not a single conv chain -- Keras Functional graphs such as
 * the EfficientNet family classify() routes by name (src/identify_tracks.py:
 * 539-540) -- as a node list in topological order.  Each node reads the
 * outputs of in0 / in1 (node indices; -1 = the model input) and writes one
 * NHWC f32 tensor per window.  The host folds BatchNormalization into a
 * preceding conv, resolves "same" padding into explicit pads and folds
 * ZeroPadding2D into the consumer's pads; activations are fused into their
 * producer where it is the only consumer.  Convs with C_in >= 16 run on the
 * runtime-shaped split-bf16 MFMA kernel (AA_PREC_BF16X3) or exact f32
 * (AA_PREC_F32); the rest is f32 VALU. */
typedef enum aa_gop {
    AA_G_CONV = 1,      /* off[0] = kernel HWIO [kh][kw][cin][filters], off[1] = bias (or -1) */
    AA_G_DWCONV = 2,    /* depthwise, depth multiplier 1: off[0] = kernel [kh][kw][C], off[1] = bias */
    AA_G_MAXPOOL = 3,   /* window kh x kw, strides, pads */
    AA_G_AVGPOOL = 4,   /* the average over the taps inside the image */
    AA_G_GMAXPOOL = 5,  /* -> [1][1][C] */
    AA_G_GAVGPOOL = 6,  /* -> [1][1][C] */
    AA_G_ADD = 7,       /* in0 + in1 (same shape) */
    AA_G_MUL = 8,       /* in0 * in1; in1 may be [1][1][C] (broadcast over H, W) */
    AA_G_AFFINE = 9,    /* x * off[0][c] + off[1][c] (standalone BatchNormalization, Rescaling,
                         * Normalization); off = -1: identity (activation only) */
    AA_G_DENSE = 10,    /* [1][1][C] (or any H x W, flattened) -> [1][1][filters]:
                         * off[0] = kernel [C][filters], off[1] = bias */
    AA_G_POW = 11,      /* x ** alpha (MagTransform: alpha = sigmoid(a)) */
} aa_gop;

typedef enum aa_gact {
    AA_GACT_NONE = 0, AA_GACT_RELU = 1, AA_GACT_LEAKY = 2, AA_GACT_SIGMOID = 3, AA_GACT_SWISH = 4
} aa_gact;

typedef struct aa_node {
    int32_t op;                  /* aa_gop */
    int32_t in0, in1;            /* producer nodes (-1: the model input; in1 unused: -1) */
    int32_t kh, kw, sh, sw;      /* window / kernel, strides */
    int32_t pt, pb, pl, pr;      /* explicit zero padding (top, bottom, left, right) */
    int32_t filters;             /* conv / dense outputs */
    int32_t act;                 /* aa_gact, applied last */
    float alpha;                 /* leaky slope (AA_G_POW: the exponent) */
    int64_t off[2];              /* weight blob offsets (floats), -1 when absent */
} aa_node;

/* The last node is the output [n][1][1][L] (or [n][H][W][L], flattened);
 * logits are its values before a sigmoid activation (equal to probs
 * otherwise). */
int aa_graph_create(const aa_node* nodes, int32_t n_nodes, const float* blob, int64_t blob_len, int32_t in_h,
                    int32_t in_w, int32_t in_c, int32_t precision, void** graph);
int aa_graph_destroy(void* graph);
int aa_graph_n_outputs(const void* graph);
size_t aa_graph_workspace_bytes(const void* graph, int32_t max_batch);
int aa_graph_forward(void* graph, const float* x, int32_t n, float* logits, float* probs, void* workspace,
                     size_t workspace_bytes, void* stream);
/* launches of one forward ("conv_gx3_*", "dwconv_*", ...), their algorithmic
 * flops / bytes per window */
int aa_graph_n_stages(const void* graph);
/* Node timing (HIP events around node launches): set_timing(mask != 0) times
 * every node, 0 none; time_stage(k) node k only (-1 every node, -2 none) --
 * a graph has more nodes than a 32-bit mask holds.  stage_time as
 * aa_model_stage_time. */
int aa_graph_set_timing(void* graph, uint32_t stage_mask);
int aa_graph_time_stage(void* graph, int32_t stage);
int aa_graph_stage_time(void* graph, int32_t stage, double* total_ms, int64_t* count);
int aa_graph_stage_info(const void* graph, int32_t stage, char* name, int32_t name_len, double* flops_per_item,
                        double* bytes_per_item);

/* ---------------- ensemble + window mean ---------------- */
/* probs: device float32, model m / window w at probs[m * model_stride + w * n_labels].
 * Track t averages windows [win_begin[t], win_begin[t] + win_count[t]) after
 * averaging over models, both in float32 with sequential accumulation like
 * numpy's axis-0 mean.  out: device float32 [n_tracks][n_labels]. */
int aa_track_mean(const float* probs, int32_t n_models, int64_t model_stride, int32_t n_labels,
                  const int32_t* win_begin, const int32_t* win_count, int32_t n_tracks,
                  float* out, void* stream);

/* ---------------------------------------------------------------- span scan */
/* flags[i] = 1 if any of pcm[spans[2i] .. spans[2i+1]) is nonzero, else 0.
 * Spans are caller-validated to lie in [0, n).  Backs get_end
 * (src/identify_tracks.py:387-413): a 170-frame chunk of the 4800/281 STFT has
 * a constant mel block exactly when every sample its frames cover is zero. */
int aa_span_nonzero(const float* pcm, int64_t n, const int64_t* spans, int32_t n_spans,
                    int32_t* flags, void* stream);

/* Device PCM16 (interleaved, `channels` <= 8) -> mono f32, as load_recording
 * delivers it (src/identify_tracks.py:49-62: ffmpeg s16, librosa buf_to_float
 * x / 32768, channel mean): bit-identical to the host decode.  Lets a batch of
 * recordings cross PCIe as int16. */
int aa_pcm_s16_to_f32(const int16_t* in, int64_t n_frames, int32_t channels, float* out, void* stream);

/* Rational polyphase resampling by L / M (load_recording's librosa.resample
 * to 48 kHz, src/identify_tracks.py:49-62; libsoxr's HQ recipe restated, see
 * aa_amd/resample.py): y[m] = sum_t bank[r][t] x[k0 - t] with q = m M + half,
 * k0 = q / L, r = q % L; x is zero outside [0, n_in).  bank: device f32
 * [L][taps] (bank[r][t] = h[r + t L] of the filter on the L-times upsampled
 * grid, centre tap `half`). */
int aa_resample_poly(const float* x, int64_t n_in, const float* bank, int32_t L, int32_t M, int32_t taps,
                     int32_t half, float* y, int64_t n_out, void* stream);

/* ---------------------------------------------------------------- signal detector */
/* signal_noise (src/identify_tracks.py:650-706): |STFT| (n_fft 4096) of the
 * recording, the 3x row/column-median mask, cv2 morphology, 8-connected
 * components and the size filter, all on the device. */
typedef struct aa_sn_config {
    int32_t sr;          /* sample rate of the PCM (48000 after load_recording) */
    int32_t n_fft;       /* 4096 (:652) */
    int32_t hop_length;  /* 281 (:420) */
    double signal_width; /* SIGNAL_WIDTH seconds (:21, :673) */
    double freq_range;   /* Hz; the first bin above it sets the kernel height (:675-681) */
} aa_sn_config;

/* One kept component: the cv2 stats row (x = frame, y = frequency bin) and
 * OpenCV's label-order key, which orders components that tie on `left` in the
 * reference's stable sort (:688). */
typedef struct aa_sn_component {
    int32_t left, top, width, height, area, order;
} aa_sn_component;

#define AA_SN_NONFINITE 1    /* status: non-finite PCM (librosa valid_audio would raise) */
#define AA_SN_RUN_OVERFLOW 2 /* status: run table bound exceeded (internal error) */

int aa_sn_create(const aa_sn_config* cfg, void** plan);
int aa_sn_destroy(void* plan);
/* {dilate height, dilate width, erode height, erode width, min width, min
 * height} as derived from cfg (:673-691); host only */
int aa_sn_geometry(const aa_sn_config* cfg, int32_t* out6);
/* STFT frames of n_samples: 1 + n_samples / hop_length */
int64_t aa_sn_n_frames(const void* plan, int64_t n_samples);
size_t aa_sn_workspace_bytes(const void* plan, int64_t max_samples);
/* pcm: device f32 [n_samples] (frames[: int(sr * length)], :420).
 * out: device aa_sn_component[max_out], unordered; n_out: device int32[2] =
 * {components kept (may exceed max_out), AA_SN_* status}.
 * mask_out (may be NULL): device uint64 [2049][ceil(F / 64)], the thresholded
 * mask before morphology; bit f % 64 of word f / 64 is frame f. */
int aa_sn_run(void* plan, const float* pcm, int64_t n_samples, void* workspace, size_t workspace_bytes,
              aa_sn_component* out, int32_t max_out, int32_t* n_out, uint64_t* mask_out, void* stream);
/* signal_noise of n_rec (1..64) recordings in one device PCM buffer in one
 * pass (the batched corpus path; the reference runs it once per file,
 * src/identify_tracks.py:420): recording k is pcm[offsets[k] ..
 * offsets[k] + lengths[k]) (offsets, lengths: HOST arrays).  Its components
 * go to out + k * out_stride (out_stride >= max_out), its {count, status} to
 * n_out + k * n_out_stride (>= 2).  The per-recording STFT / medians / mask
 * launches run back to back; the morphology and components run once for the
 * whole batch.  Workspace: aa_sn_batch_workspace_bytes(plan, longest, n_rec). */
size_t aa_sn_batch_workspace_bytes(const void* plan, int64_t max_samples, int32_t n_rec);
int aa_sn_run_batch(void* plan, const float* pcm, const int64_t* offsets, const int64_t* lengths, int32_t n_rec,
                    void* workspace, size_t workspace_bytes, aa_sn_component* out, int32_t max_out,
                    int64_t out_stride, int32_t* n_out, int32_t n_out_stride, void* stream);
/* np.abs(librosa.stft(pcm, n_fft=4096, hop_length=hop)) (:654) alone, in the
 * reference's precision (f64 transform, complex64 rounding, numpy's f32
 * magnitude): out = device f32 [F][ld] (F = aa_sn_n_frames, ld >= 2049), row f
 * = frame f's 2049 bins.  No workspace. */
int aa_sn_spectrogram(void* plan, const float* pcm, int64_t n_samples, float* out, int64_t ld, void* stream);
/* Launch stages of aa_sn_run / aa_sn_run_batch (0 sn_stft64, 1 sn_transpose,
 * 2 sn_select, 3 sn_morph, 4 the component launches, 5 sn_colmed) and their timing, the
 * aa_fe_stage_* contract; an item is one STFT frame of one recording. */
int aa_sn_n_stages(const void* plan);
int aa_sn_stage_info(const void* plan, int32_t stage, char* name, int32_t name_len, double* flops_per_item,
                     double* bytes_per_item);
int aa_sn_set_timing(void* plan, uint32_t stage_mask);
int aa_sn_stage_time(void* plan, int32_t stage, double* total_ms, int64_t* count);
/* Morphology, components and filter of a given mask (mask_out's layout). */
int aa_sn_components_from_mask(void* plan, const uint64_t* mask, int64_t n_frames, void* workspace,
                               size_t workspace_bytes, aa_sn_component* out, int32_t max_out,
                               int32_t* n_out, void* stream);

/* ---------------------------------------------------------------- FLAC decode */
/* load_recording (src/identify_tracks.py:49-62) decodes through ffmpeg; these
 * decode a FLAC stream (RFC 9639; an ID3v2 tag in front is skipped) held in
 * HOST memory, on the calling thread.  Samples come out as the stream's own
 * integers (bits_per_sample), interleaved; the caller applies ffmpeg's s16
 * conversion.  Header CRC-8 and frame CRC-16 are verified (AA_ERR_INVALID on
 * damage, with the byte offset in aa_last_error). */
typedef struct aa_flac_stream_info {
    int32_t sample_rate;
    int32_t channels;        /* 1..8 */
    int32_t bits_per_sample; /* 4..32 */
    int64_t total_frames;    /* samples per channel; 0 = not stated */
} aa_flac_stream_info;

int aa_flac_info(const uint8_t* data, size_t len, aa_flac_stream_info* info);
/* out: host int32 [cap_frames][channels], or NULL to count only;
 * n_frames: frames (samples per channel) decoded.  AA_ERR_WORKSPACE when the
 * stream holds more than cap_frames. */
int aa_flac_decode(const uint8_t* data, size_t len, int32_t* out, int64_t cap_frames, int64_t* n_frames);

/* ---------------------------------------------------------- Ogg Vorbis decode */
/* load_recording (src/identify_tracks.py:49-62) decodes through ffmpeg; these
 * decode an Ogg Vorbis stream (RFC 3533 pages, Vorbis I codec: floor 0/1,
 * residue 0/1/2, channel coupling, short/long blocks) held in HOST memory, on
 * the calling thread.  Pages failing their CRC-32 are skipped; the first
 * Vorbis logical stream is decoded.  Samples come out as float32 in [-1, 1]
 * scale, interleaved, trimmed by the granule positions (Vorbis I A.2); the
 * caller applies ffmpeg's float -> s16 conversion.  A damaged header is
 * AA_ERR_INVALID with the reason in aa_last_error. */
typedef struct aa_vorbis_stream_info {
    int32_t sample_rate;
    int32_t channels;        /* 1..255 */
    int32_t blocksize_0;     /* short block, 64..8192 */
    int32_t blocksize_1;     /* long block */
    int64_t total_frames;    /* the last page's granule position (0 = none found) */
} aa_vorbis_stream_info;

int aa_vorbis_info(const uint8_t* data, size_t len, aa_vorbis_stream_info* info);
/* out: host float32 [cap_frames][channels], or NULL to count only;
 * n_frames: frames (samples per channel) decoded.  AA_ERR_WORKSPACE when the
 * stream holds more than cap_frames. */
int aa_vorbis_decode(const uint8_t* data, size_t len, float* out, int64_t cap_frames, int64_t* n_frames);

/* ---- file input of the batched corpus path (aa_amd/batch.py) ----
 * The whole file at path into buf (cap bytes; a pinned staging slot), in one
 * call: open, size, read, close -- the reference reads each file through
 * ffmpeg (src/identify_tracks.py:49-62); the corpus decoder threads read
 * PCM16 WAVs raw and parse the RIFF header themselves.  *size: the file's
 * size.  AA_ERR_WORKSPACE (nothing read) when it exceeds cap;
 * AA_ERR_INVALID when it cannot be opened or read (the reason in
 * aa_last_error). */
int aa_read_file(const char* path, void* buf, int64_t cap, int64_t* size);

/* ---- track builder (host) ----
 * get_tracks_from_signals (src/identify_tracks.py:795-842, with
 * merge_signals :725-792): the signals' merge sweeps until stable, then the
 * enlarge / absorb pass and the narrow-track drop, in Python's double
 * arithmetic.  sig: n rows of (start, end, freq_start, freq_end,
 * mel_freq_start, mel_freq_end); kind: per row, which of the first four are
 * Python ints (bits 0-3: start, end, freq_start, freq_end).  end: the
 * recording's length (end_is_int: a Python int).  mel_int[f]: the mel of
 * integer frequency f (numpy's 2595 log10(1 + f / 700)), n_mel entries.
 * Out: *n_tracks rows (<= n) of the same layout into track / track_kind.
 * AA_ERR_INVALID where the Python divides by a zero mel range (it raises
 * there); AA_ERR_UNSUPPORTED when an enlarged frequency is outside mel_int or
 * an input is NaN (the caller's Python builder takes those). */
int aa_tracks_from_signals(const double* sig, const int32_t* kind, int64_t n, double end, int32_t end_is_int,
                           const double* mel_int, int64_t n_mel, double* track, int32_t* track_kind,
                           int64_t* n_tracks);

#ifdef __cplusplus
}
#endif
#endif /* AA_H */
