/*
 * pss_hip.h -- C ABI of libpss_hip.so, the MI355X (gfx950) engine behind
 * PsrSigSim's filterbank synthesis path.
 *
 * The reference has no FFI: its boundary is the Python method API (SURVEY.md
 * §8(b)).  Each entry point below replaces one reference call (or a fused run
 * of several), cited file:line against /root/reference/psrsigsim.  The Python
 * layer (psrsigsim_amd, ctypes) mirrors the reference classes and calls these.
 *
 * Conventions
 *  - All buffers are DEVICE pointers owned by the caller (torch); the library
 *    never allocates or frees user memory.  Row-major [chan][sample] fp32.
 *  - Every call is stream-ordered on `stream` (a hipStream_t; NULL = default)
 *    and performs no host synchronisation; it is graph-capturable.
 *  - Return codes: PSS_OK = 0, PSS_EINVAL = -1 (-> ValueError),
 *    PSS_EUNSUPPORTED = -2 (-> NotImplementedError), PSS_EHIP = -3
 *    (-> RuntimeError); pss_last_error() returns the message.
 *  - Randomness is counter-based Philox4x32-7 keyed by (seed, call id,
 *    purpose, GLOBAL channel, sample): results do not depend on how channels
 *    are split across launches or GPUs.
 */
#ifndef PSS_HIP_H
#define PSS_HIP_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PSS_OK 0
#define PSS_EINVAL (-1)
#define PSS_EUNSUPPORTED (-2)
#define PSS_EHIP (-3)

/* source of the real (data) part */
#define PSS_SRC_LOAD 0   /* read `data` (an already materialised signal)       */
#define PSS_SRC_SEARCH 1 /* pulsar.py:222-244 PCHIP(phase) x chi2(df) x norm    */
#define PSS_SRC_FOLD 2   /* pulsar.py:196-221 tile(profile) x chi2(Nfold) x norm */

/* null stage */
#define PSS_NULL_NONE 0
#define PSS_NULL_UNDELAYED 1 /* pulsar.py:292-304: replace boxes, shared vector  */
#define PSS_NULL_DELAYED 2   /* pulsar.py:306-330: chi2(100) box mask shifted
                                through the same FFT, thresholded > 1           */

/* observe() copy ("out") dtypes */
#define PSS_OUT_NONE 0
#define PSS_OUT_F32 1
#define PSS_OUT_I8 2

/*
 * One fused run of the synthesis path over `nchan` rows:
 *
 *   source  ->  [delay ramp: rfft -> exp(-2 pi i f tau) -> irfft]  ->  [null]
 *           ->  [radiometer noise]  ->  data      (+ optional pre-noise `out`)
 *
 * Replaces, for one signal, the sequence
 *   Pulsar.make_pulses        pulsar/pulsar.py:107-151,185-244
 *   ISM.disperse / FD_shift / scatter_broaden(convolve=False)
 *                             ism/ism.py:20-74, 100-156, 158-220
 *                             (each = per-channel utils.shift_t, utils/utils.py:17-59)
 *   Pulsar.null               pulsar/pulsar.py:246-333
 *   Telescope.observe (copy branch) + Receiver.radiometer_noise
 *                             telescope/telescope.py:72-149, receiver.py:82-172
 * with any prefix/subset of the stages enabled.  Several delay stages are
 * fused into one forward/inverse FFT pair: phase exp(-2 pi i k sum(s_j)/N) on
 * every bin, and on the Nyquist bin the product of the per-stage factors
 * cos(pi s_j) that the reference's irfft imposes.
 */
typedef struct PssPipeline {
    /* geometry */
    int32_t nchan;      /* rows in this launch                                  */
    int32_t chan0;      /* global channel index of row 0 (RNG key, table rows)  */
    int64_t nsamp;      /* N: samples per row (= data.shape[1])                */
    int64_t ld;         /* row stride of `data` in elements                     */
    float *data;        /* [nchan][ld] in/out                                   */
    void *work;         /* workspace, >= pss_workspace_bytes(nchan, nsamp)      */

    /* source */
    int32_t src;        /* PSS_SRC_*                                            */
    int32_t prof_rows;  /* rows of `prof` (1 = same profile for every channel)  */
    const float *prof;  /* SEARCH: [prof_rows][nint][4] PCHIP coefficients in the
                           local interval coordinate u in [0,1): c3 u^3+c2 u^2+c1 u+c0
                           FOLD: [prof_rows][nph] profile samples              */
    int32_t nint;       /* SEARCH: number of PCHIP intervals                    */
    int32_t nph;        /* FOLD: phase bins per period; NULL: box length        */
    uint64_t phase_step;/* SEARCH: 2^64 / (samples per period), i.e. the pulse
                           phase advance per sample in 2^-64 cycles             */
    uint32_t knot_m;    /* SEARCH: 1/knot spacing (intervals per cycle)         */
    float gen_df;       /* chi2 degrees of freedom of the pulse draws           */
    float draw_norm;    /* signal._draw_norm                                    */

    /* delay ramp (fused delay stages) -- all arrays indexed by local row       */
    int32_t shift;          /* 1: run the FFT delay engine                     */
    int32_t data_in_fft;    /* 1: real part carries the data through the FFT;
                               0: the epilogue reads `data` unshifted (only the
                               null mask goes through the FFT)                  */
    const uint64_t *ramp;   /* [nchan] frac(s/N) in 2^-64 cycles, s = total delay
                               in samples: bin k gets exp(-2 pi i k' s / N)     */
    const float *nyq_re;    /* [nchan] Nyquist factor for the real part         */
    const float *nyq_im;    /* [nchan] Nyquist factor for the imaginary part    */

    /* null */
    int32_t null_mode;      /* PSS_NULL_*                                       */
    int32_t null_slots;     /* length of null_rank (= nsub)                     */
    const int32_t *null_rank;  /* [null_slots] order of the nulled pulse in the
                               reference's np.random.choice list, or -1         */
    int64_t null_shift;     /* shift_val (pulsar.py:286)                        */
    float null_box_df;      /* chi2 df of the box values (mask / undelayed)     */
    float null_box_scale;   /* box scale: draw_norm (mask) or draw_norm*opm     */
    float null_rep_df;      /* DELAYED: df of the replacement draws             */
    float null_rep_scale;   /* DELAYED: draw_norm * off-pulse mean              */

    /* radiometer noise */
    int32_t noise;          /* 1: data += noise_norm * chi2(noise_df)           */
    float noise_df;
    float noise_norm;

    /* observe() pre-noise copy */
    int32_t out_kind;       /* PSS_OUT_*                                        */
    void *out;              /* [nchan][nsamp] float32 or int8                   */
    float clip;             /* out = min(pre-noise, clip) (telescope.py:140-145)*/

    /* randomness */
    uint64_t seed;
    uint32_t call_gen;      /* call ids: one per API call that drew randomness  */
    uint32_t call_null;     /* (make_pulses / null / noise), so that repeated   */
    uint32_t call_noise;    /* calls draw fresh values, like np.random          */

    /* exact mode: injected draws (NULL = use Philox) */
    const float *inj_gen;     /* [nchan][nsamp] pulse chi2 draws                */
    const float *inj_box;     /* [nsamp] box values (already scaled), shared    */
    const float *inj_rep;     /* [nchan][nsamp] DELAYED replacement values      */
    const float *inj_noise;   /* [nchan][nsamp] noise chi2 draws                */

    /* DELAYED null: [nchan] frac(s_mask/N) in 2^-64 cycles, s_mask = the
       signal's total delay in samples (pulsar.py:322-325).  Four-step lengths
       (N = 2^m >= 2^14) decide mask > 1 from a once-per-run table of the box
       row shifted by the fraction of s_mask; the other
       lengths use `ramp`/`nyq_im` and carry the mask through the FFT.       */
    const uint64_t *mask_ramp;

    /* Baseband path (ISM._disperse_baseband ism/ism.py:76-98,
       Pulsar._make_amp_pulses pulsar/pulsar.py:153-183).                     */
    int32_t gen_amp;        /* SEARCH source: sqrt(profile) x N(0,1) draws
                               (amplitude pulses) instead of profile x chi2;
                               1: PCHIP table, 2: analytic Gaussians, prof =
                               [nint][4] {peak, 1/width, amp/Amax, 0} and
                               knot_m = 1 (portraits.py:277-290)             */
    int32_t prof_row0;      /* global channel of `prof`'s row 0 when the table
                               holds a channel window (shard-local planning):
                               channel c reads row c - prof_row0; 0 for a
                               band-wide table (ignored when prof_rows == 1)  */
    const float *htab;      /* [nsamp/2 + 1] complex64 transfer function H(k)
                               of the reference's rfft bins (same for every
                               row): bin k gets H(k), bin N-k conj H(k), DC
                               and Nyquist Re H (irfft drops their imaginary
                               parts).  Non-NULL: replaces the delay ramp and
                               takes the direct / Bluestein transforms.      */
    const int64_t *null_shift_dev;  /* NULL: use null_shift; else the device
                               word pss_null_shift wrote (shift_val computed on
                               the device, no host round trip)                */
    const float *tail_a;    /* [nchan] scattering tail (extension, no reference
                               counterpart -- SURVEY App. A.11): circular
                               convolution of each row with the normalised
                               exponential h[n] = (1-a) a^n, a = exp(-dt/tau_c),
                               i.e. bin k x H(k) = (1-a) / (1 - a e^{-2 pi i k/N})
                               in the same forward/inverse pass as the delay
                               ramp; NULL = none                             */
    int32_t prof_split;     /* SEARCH: 1 = `prof` holds split cells for a portrait
                               on non-uniform phases: [prof_rows][nint][8]
                               (the cubics left and right of the cell's one
                               interior knot, in the cell coordinate u) followed
                               by [nint] split points (u >= split: right cubic;
                               2 = no knot in the cell); knot_m = nint cells */
    /* observe()'s RESAMPLED pre-noise copy, produced by the run itself
       (telescope.py:108-125 down_sample / rebin, then :140-145 clip and cast):
       out_len > 0 makes `out` [nchan][out_len] of kind out_kind, bin i = the
       mean of the pre-noise samples [lo_i, hi_i), clipped from above at `clip`.
       Every epilogue adds its samples' values into out_acc (float64 window
       sums, zeroed by pss_run), a final small kernel divides, clips and casts:
       no full-resolution copy, no separate resampling pass.                 */
    int32_t out_len;        /* 0: `out` is the full [nchan][nsamp] copy         */
    const int64_t *out_lo;  /* [out_len] window starts (utils.py:77-89's ceil
                               edges), or NULL: uniform windows of out_step
                               samples, lo_i = i * out_step (down_sample,
                               utils.py:62-68)                                 */
    const int64_t *out_hi;  /* [out_len] window ends (exclusive), or NULL       */
    double out_step;        /* nominal window width: the bin of sample n is
                               floor(n / out_step) or the one before it; an
                               integer >= 1 when out_lo is NULL               */
    double *out_acc;        /* [nchan][out_len] float64 scratch                 */
} PssPipeline;

/* Library / device info. */
int pss_version(void);
/* "PSS_BUILD_HASH=<sha256 of the sources the library was built from>". */
const char *pss_build_hash(void);

/* Engine flags (test hook; returns the previous flags).  PSS_FLAG_NO_FAST
 * routes every run through the generic kernels instead of the fast-path
 * specialisations (which must give bitwise identical results). */
#define PSS_FLAG_NO_FAST 1
/* PSS_FLAG_DIRECT_DFT sends the fallback lengths N > 8192 through the O(N^2)
 * direct DFT instead of the Bluestein (chirp-z) path (test hook). */
#define PSS_FLAG_DIRECT_DFT 2
/* PSS_FLAG_NULL_F32 keeps the packed (direct / Bluestein) paths' delayed-null
   decisions in fp32 (no float64 re-evaluation near the threshold).          */
#define PSS_FLAG_NULL_F32 4
/* PSS_FLAG_REFINE_PER_SAMPLE runs those float64 re-evaluations through the
   per-sample kernel instead of the compacted candidate list (the list's
   overflow path; test hook: both give the same bits).                      */
#define PSS_FLAG_REFINE_PER_SAMPLE 8
int pss_set_flags(int flags);
int pss_last_error(char *buf, size_t n);

/* Launch-plan log (test hook): the kernels every pss_run since the last call
 * picked, one line per run -- "<nchan>x<nsamp>: <path> <split> A:<pass A>
 * R:<row pass> C:<pass C> N:<null>", e.g. "2048x4194304: fourstep 1024x4096
 * A:fast R:pair_row C:fast N:table N:fix_list" -- copied into buf (up to n - 1
 * bytes, NUL-terminated); returns the log's length and clears it.  The parity
 * tests assert with it which kernels produced the bits they check.        */
int pss_plan_collect(char *buf, size_t n);

/* Opt-in kernel timing for benchmarks: while enabled, pss_run records a pair
 * of hipEvents on its stream around every kernel it launches.  collect()
 * synchronises on them and returns, per launch (up to `cap`), the kernel kind
 * (0 elementwise, 1 single pass, 2 four-step column pass A, 3 row pass B,
 * 4 column pass C, 5 fallback, 6 delayed-null fix-up), its milliseconds and the channel-samples it
 * processed; returns the number of launches reported and resets. */
void pss_timing_enable(int on);
int pss_timing_collect(int32_t *kind, double *ms, int64_t *units, int cap);
/* Milliseconds from the start of the first timed launch to the end of the
 * last one since the last collect (the device span of the runs: with pair
 * batches on side streams the per-kernel times overlap). */
double pss_timing_span_ms(void);

/* Workspace bytes the fused run needs for `nchan` rows of length `nsamp`. */
int64_t pss_workspace_bytes(int32_t nchan, int64_t nsamp);

/* The fused run (see PssPipeline). */
int pss_run(const PssPipeline *p, void *stream);

/*
 * utils.shift_t on a batch of rows (utils/utils.py:17-59): every row r is
 * shifted by shift_samples[r] (= shift/dt, may be fractional) through the same
 * FFT engine.  `nyq` is the Nyquist factor per row (cos(pi*s) for one
 * reference call; unused for odd N).  In place.  Odd N (3 <= N <= 2^20): the
 * reference's irfft without n= returns N-1 samples (utils.py:57); they are
 * written to the first N-1 columns of each row (direct DFTs, f64 sums).
 */
/* Filter rows by a per-bin transfer function (baseband coherent dispersion,
 * ism/ism.py:76-98): rows <- irfft(rfft(row) * H) in place, H = htab
 * [n/2 + 1] complex64 (interleaved re, im).  Even n <= 2^24.  Workspace:
 * pss_filter_workspace_bytes(nrows, n). */
int64_t pss_filter_workspace_bytes(int32_t nrows, int64_t n);
int pss_filter_rows(float *rows, int32_t nrows, int64_t n, int64_t ld, const float *htab,
                    void *work, void *stream);

int pss_shift_rows(float *rows, int32_t nrows, int64_t n, int64_t ld,
                   const uint64_t *ramp, const float *nyq, void *work, void *stream);

/* utils.down_sample per row (utils/utils.py:62-68): out[r][i] = mean of
 * in[r][i*fact : (i+1)*fact]; in_len must be a multiple of fact. */
int pss_down_sample(const float *in, float *out, int32_t nrows, int64_t in_len,
                    int64_t in_ld, int32_t fact, void *stream);

/* utils.rebin per row (utils/utils.py:71-91): `lo`/`hi` are the integer window
 * edges [lo_i, hi_i) the reference derives from its ceil() arithmetic, device
 * arrays of `newlen` entries with 0 <= lo_i <= hi_i <= in_len (not checked:
 * they live on the device).  PSS_EINVAL on NULL pointers or in_ld < in_len. */
int pss_rebin(const float *in, float *out, int32_t nrows, int64_t in_len, int64_t in_ld,
              int32_t newlen, const int64_t *lo, const int64_t *hi, void *stream);

/* Telescope.observe tail (telescope.py:140-145): clip from above at `clip`,
 * cast to float32 or int8 (truncation toward zero, as numpy's astype). */
int pss_clip_cast(const float *in, void *out, int64_t count, float clip, int32_t out_kind,
                  void *stream);

/* Backend.fold (telescope/backend.py:34-49): out[c][b] =
 * sum_{f<n_fold} data[c][npbins + f*half + b], half = npbins/2. */
int pss_fold(const float *data, float *out, int32_t nchan, int64_t ld, int64_t npbins,
             int64_t n_fold, void *stream);

/* Corrected fold (extension, no reference
 * counterpart -- backend.py:34-49 is only valid for exactly four periods):
 * out[c][b] = sum_{p<nper} data[c][p*nbin + b] over whole periods of `nbin`
 * samples, float64 accumulation, float32 out. */
int pss_fold_periods(const float *data, float *out, int32_t nchan, int64_t ld, int64_t nbin,
                     int64_t nper, void *stream);

/*
 * Native host planning (no GPU; bitwise replicas of the float64 NumPy
 * arithmetic in psrsigsim_amd/pulsar/portraits.py, itself pinned to the
 * reference's scipy PCHIP -- pulsar/portraits.py:200-267 of the reference).
 * `nthreads` host threads split the rows.
 *   pss_host_pchip_coef:   c[rows][K-1][4] piecewise-cubic coefficients
 *                          (powers 3..0 of t - x_i) through y[rows][K] at x[K]
 *   pss_host_ppoly_eval:   out[rows][n] = the cubic at phases ph[n]
 *                          (interval = last x_i <= phase, end pieces extrapolate)
 *   pss_host_device_table: out[rows][nint][4] (float32) = c * (h^3, h^2, h, 1)
 *                          / amax (the table the source stage evaluates)
 *   pss_host_pchip_eval:   pchip_coef then ppoly_eval (then / div when div != 1)
 *                          fused per row: no coefficient table in memory
 *   pss_host_pchip_table:  pchip_coef then device_table fused per row (hcell = h)
 */
int pss_host_pchip_coef(const double *x, int64_t K, const double *y, int64_t rows, double *c,
                        int nthreads);
int pss_host_ppoly_eval(const double *x, int64_t K, const double *c, int64_t rows, const double *ph,
                        int64_t n, double *out, int nthreads);
int pss_host_device_table(const double *c, int64_t rows, int64_t nint, double h, double amax,
                          float *out, int nthreads);
int pss_host_pchip_eval(const double *x, int64_t K, const double *y, int64_t rows, const double *ph, int64_t n,
                        double div, double *out, int nthreads);
int pss_host_pchip_table(const double *x, int64_t K, const double *y, int64_t rows, double hcell, double amax,
                         float *out, int nthreads);

/* Pulsar.null's shift_val (pulsar/pulsar.py:285-288) on the device:
 *   shift_val = count / 2 - argmax(row[0:count])
 * out[0] = shift_val (int64), out[1] = status: 0 ok; 1 the maximum is not
 * unique; 2 a NaN in the row (the reference's np.where then yields 0 or >1
 * indices and the broadcast raises ValueError).  Stream-ordered, no host
 * synchronisation: the fused run reads out[0] through
 * PssPipeline.null_shift_dev. */
int pss_null_shift(const float *row, int64_t count, int64_t *out, void *stream);

/* Philox chi2 draws (test hook + CPU-independent statistics checks):
 * out[r][n] = chi2(df) keyed like the pipeline's purpose `purpose`. */
int pss_chi2_fill(float *out, int32_t nrows, int32_t chan0, int64_t n, float df,
                  uint64_t seed, uint32_t call_id, uint32_t purpose, void *stream);


#ifdef __cplusplus
}
#endif
#endif /* PSS_HIP_H */
