// pss_host.cpp -- native host planning for the profile-level tables.
//
// The profile tables the device path evaluates (PCHIP coefficients of every
// channel's portrait, their evaluation at resampling phases, the float32
// device table) are O(Nchan x Nph) float64 work done once per signal on the
// host.  The NumPy formulation spends its time on (Nchan x Nph) temporaries
// (page faults, memory traffic); these loops do one pass per row, spread over
// host threads, with EXACTLY the operations and order of the NumPy code they
// replace (psrsigsim_amd/pulsar/portraits.py: pchip_coefficients, ppoly_eval,
// DataPortrait.device_table), so results are bitwise identical -- the reference
// makes exact float decisions on these values (portraits.py:234).
//
// No FMA contraction anywhere in this file (numpy evaluates each binary op
// separately in IEEE double).
#pragma clang fp contract(off)

#include <math.h>
#include <stdint.h>
#include <string.h>

#include <unistd.h>

#include <algorithm>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/pss_hip.h"

namespace {

// np.sign as a double: -1, 0, +1, NaN for NaN
inline double sgn(double v) { return v > 0.0 ? 1.0 : (v < 0.0 ? -1.0 : (v == 0.0 ? 0.0 : v)); }

// portraits.py _edge_slope (scipy's one-sided three-point end slope + clamps)
inline double edge_slope(double h0, double h1, double m0, double m1) {
    double d = ((2.0 * h0 + h1) * m0 - h0 * m1) / (h0 + h1);
    const bool flip = sgn(d) != sgn(m0);          // NaN compares unequal, as in numpy
    const bool big = (sgn(m0) != sgn(m1)) && (fabs(d) > 3.0 * fabs(m0));
    if (flip) d = 0.0;
    return (!flip && big) ? 3.0 * m0 : d;
}

// A persistent pool of host threads for the row passes: starting and joining
// std::threads costs ~20-100 us each per call, more than a share of these
// passes on a 2048-row table (two or three calls per signal).  Workers are
// started once (lazily, and again in a forked child: the pool records its
// pid), then wait for row blocks.
class Pool {
  public:
    void run(int64_t rows, int nt, const std::function<void(int64_t, int64_t)> &fn) {
        std::lock_guard<std::mutex> one(run_mu_);   // one pass at a time (callers on several threads)
        std::unique_lock<std::mutex> lk(mu_);
        ensure(nt - 1);
        fn_ = &fn;
        rows_ = rows;
        nt_ = nt;
        next_ = 1;                     // block 0 runs on the calling thread
        done_ = 0;
        ++gen_;
        cv_.notify_all();
        lk.unlock();
        fn(0, rows / nt);
        lk.lock();
        done_cv_.wait(lk, [&] { return done_ == nt_ - 1; });
        fn_ = nullptr;
    }

  private:
    void ensure(int workers) {
        if (pid_ != getpid()) {        // a forked child: the parent's workers do not exist here
            for (auto &t : th_) t.detach();
            th_.clear();
            pid_ = getpid();
        }
        while ((int)th_.size() < workers) th_.emplace_back([this] { loop(); });
    }
    void loop() {
        uint64_t seen = 0;
        std::unique_lock<std::mutex> lk(mu_);
        const pid_t me = pid_;
        for (;;) {
            cv_.wait(lk, [&] { return gen_ != seen && fn_ && next_ < nt_; });
            if (pid_ != me) return;
            const int b = next_++;
            if (next_ >= nt_) seen = gen_;
            const int64_t a = rows_ * b / nt_, e = rows_ * (b + 1) / nt_;
            const std::function<void(int64_t, int64_t)> *fn = fn_;
            lk.unlock();
            (*fn)(a, e);
            lk.lock();
            if (++done_ == nt_ - 1) done_cv_.notify_one();
        }
    }
    std::mutex run_mu_, mu_;
    std::condition_variable cv_, done_cv_;
    std::vector<std::thread> th_;
    const std::function<void(int64_t, int64_t)> *fn_ = nullptr;
    int64_t rows_ = 0;
    int nt_ = 0, next_ = 0, done_ = 0;
    uint64_t gen_ = 0;
    pid_t pid_ = 0;
};

Pool &pool() {
    static Pool *p = new Pool();       // (never destroyed: workers may outlive static teardown)
    return *p;
}

template <typename F>
void parallel_rows(int64_t rows, int nthreads, F fn) {
    if (nthreads <= 1 || rows < 512) {
        fn(0, rows);
        return;
    }
    // >= 256 rows per block (make_pulses at 256 channels x 244 phases: one
    // block on one thread beats splitting it)
    const int nt = (int)std::min<int64_t>(nthreads, rows / 256);
    if (nt <= 1) {
        fn(0, rows);
        return;
    }
    const std::function<void(int64_t, int64_t)> f = fn;
    pool().run(rows, nt, f);
}

}  // namespace

extern "C" {

}  // extern "C"

namespace {

// The PCHIP coefficients of the intervals [a, b) of one row (0 <= a < b <=
// K - 1): the NumPy statement's operations restricted to that range (secants
// m over [a - 1, b], slopes d over [a, b]), so a row cut into spans gives the
// bits of the whole-row pass.  mm / dd: scratch of >= b - a + 2 and b - a + 1;
// cr receives (b - a) x 4.  The interior slope is computed on flat knots too
// and then discarded (a select instead of a branch, so the loop vectorises;
// the kept values are the same operations).
inline void pchip_span(const double *h, int64_t K, const double *yr, int64_t a, int64_t b, double *mm,
                       double *dd, double *cr) {
    const int64_t ma = a > 0 ? a - 1 : 0, mb = std::min<int64_t>(b + 1, K - 1);
    for (int64_t i = ma; i < mb; ++i) mm[i - ma] = (yr[i + 1] - yr[i]) / h[i];
    if (K == 2) {
        dd[0] = dd[1] = mm[0];
    } else {
        const int64_t ia = std::max<int64_t>(a, 1), ib = std::min<int64_t>(b, K - 2);
        for (int64_t i = ia; i <= ib; ++i) {
            const double m0 = mm[i - 1 - ma], m1 = mm[i - ma];
            const double w1 = 2.0 * h[i] + h[i - 1];
            const double w2 = h[i] + 2.0 * h[i - 1];
            const bool flat = (std::signbit(m0) != std::signbit(m1)) || (m1 == 0.0) || (m0 == 0.0);
            const double v = 1.0 / ((w1 / m0 + w2 / m1) / (w1 + w2));
            dd[i - a] = flat ? 0.0 : v;
        }
        if (a == 0) dd[0] = edge_slope(h[0], h[1], mm[0 - ma], mm[1 - ma]);
        if (b == K - 1) dd[b - a] = edge_slope(h[K - 2], h[K - 3], mm[K - 2 - ma], mm[K - 3 - ma]);
    }
    for (int64_t i = a; i < b; ++i) {
        const double d0 = dd[i - a], d1 = dd[i + 1 - a], hi = h[i], mi = mm[i - ma];
        const double t = (d0 + d1 - 2.0 * mi) / hi;
        double *c = cr + 4 * (i - a);
        c[0] = t / hi;
        c[1] = (mi - d0) / hi - t;
        c[2] = d0;
        c[3] = yr[i];
    }
}

// One row's PCHIP coefficients: m, d scratch of K - 1 and K; cr (K - 1) x 4.
inline void pchip_row(const double *h, int64_t K, const double *yr, double *m, double *d, double *cr) {
    pchip_span(h, K, yr, 0, K - 1, m, d, cr);
}

// Per-thread scratch rows (reused across calls: no allocation per row).
inline double *scratch(int which, int64_t n) {
    static thread_local std::vector<double> buf[3];
    if ((int64_t)buf[which].size() < n) buf[which].resize(n);
    return buf[which].data();
}

// fn(r, a, b) over spans [a, b) of the K - 1 intervals of each of `rows`
// rows, on the host threads when there is enough work (as parallel_rows:
// >= 256 rows per block for a many-row table; a few long rows -- a 48 828-
// phase tutorial profile -- are cut into spans of >= 4096 intervals).
template <typename F>
void parallel_spans(int64_t rows, int64_t K, int nthreads, F fn) {
    const int64_t nint = K - 1;
    int64_t S = 1;
    int nt = 1;
    if (nthreads > 1 && rows >= nthreads) {
        nt = rows >= 512 ? (int)std::min<int64_t>(nthreads, rows / 256)
                         : (rows * nint >= 131072 ? nthreads : 1);   // (256 x 244: one thread is faster)
    } else if (nthreads > 1 && rows >= 1) {
        S = std::max<int64_t>(1, std::min<int64_t>((nthreads + rows - 1) / rows, nint / 4096));
        nt = (int)std::min<int64_t>(nthreads, rows * S);
        if (S == 1) nt = 1;
    }
    const int64_t tasks = rows * S;
    const std::function<void(int64_t, int64_t)> f = [&](int64_t t0, int64_t t1) {
        for (int64_t t = t0; t < t1; ++t) {
            const int64_t r = t / S, q = t % S;
            fn(r, nint * q / S, nint * (q + 1) / S);
        }
    };
    if (nt <= 1) f(0, tasks);
    else pool().run(tasks, nt, f);
}

// interval = last breakpoint <= phase (searchsorted 'right' - 1), clipped to
// the end pieces; s = phase - x[i]
inline void locate(const double *x, int64_t K, const double *ph, int64_t n, int64_t *iv, double *s) {
    for (int64_t j = 0; j < n; ++j) {
        int64_t i = (int64_t)(std::upper_bound(x, x + K, ph[j]) - x) - 1;
        i = std::min<int64_t>(std::max<int64_t>(i, 0), K - 2);
        iv[j] = i;
        s[j] = ph[j] - x[i];
    }
}

// scipy's PPoly power accumulation (lowest power first)
inline double ppoly_at(const double *ci, double sj) {
    double res = ci[3] * 1.0;
    double z = sj;
    res = res + ci[2] * z;
    z = z * sj;
    res = res + ci[1] * z;
    z = z * sj;
    res = res + ci[0] * z;
    return res;
}

}  // namespace

extern "C" {

int pss_host_pchip_coef(const double *x, int64_t K, const double *y, int64_t rows, double *c,
                        int nthreads) {
    if (K < 2 || rows < 0 || !x || !y || !c) return PSS_EINVAL;
    std::vector<double> h(K - 1);
    for (int64_t i = 0; i + 1 < K; ++i) h[i] = x[i + 1] - x[i];
    parallel_spans(rows, K, nthreads, [&](int64_t r, int64_t a, int64_t b) {
        double *m = scratch(0, b - a + 2), *d = scratch(1, b - a + 1);
        pchip_span(h.data(), K, y + r * K, a, b, m, d, c + (r * (K - 1) + a) * 4);
    });
    return PSS_OK;
}

// The PCHIP through rows of y at knots x evaluated at phases ph, divided by
// `div` when div != 1 -- pss_host_pchip_coef then pss_host_ppoly_eval then
// the division, fused per row (no [rows, K - 1, 4] coefficient table in
// memory): the same operations, so the same bits.
int pss_host_pchip_eval(const double *x, int64_t K, const double *y, int64_t rows, const double *ph, int64_t n,
                        double div, double *out, int nthreads) {
    if (K < 2 || rows < 0 || n < 0 || !x || !y || !ph || !out) return PSS_EINVAL;
    std::vector<double> h(K - 1);
    for (int64_t i = 0; i + 1 < K; ++i) h[i] = x[i + 1] - x[i];
    std::vector<int64_t> iv(n);
    std::vector<double> s(n);
    locate(x, K, ph, n, iv.data(), s.data());
    const bool dv = div != 1.0;
    parallel_rows(rows, nthreads, [&](int64_t r0, int64_t r1) {
        std::vector<double> m(K - 1), d(K), cr((K - 1) * 4);
        for (int64_t r = r0; r < r1; ++r) {
            pchip_row(h.data(), K, y + r * K, m.data(), d.data(), cr.data());
            double *o = out + r * n;
            for (int64_t j = 0; j < n; ++j) {
                const double v = ppoly_at(cr.data() + 4 * iv[j], s[j]);
                o[j] = dv ? v / div : v;
            }
        }
    });
    return PSS_OK;
}

// DataPortrait.device_table straight from the knot values: pss_host_pchip_coef
// then pss_host_device_table, fused per row (the same operations and bits).
int pss_host_pchip_table(const double *x, int64_t K, const double *y, int64_t rows, double hcell, double amax,
                         float *out, int nthreads) {
    if (K < 2 || rows < 0 || !x || !y || !out) return PSS_EINVAL;
    std::vector<double> h(K - 1);
    for (int64_t i = 0; i + 1 < K; ++i) h[i] = x[i + 1] - x[i];
    const double w[4] = {pow(hcell, 3.0), pow(hcell, 2.0), hcell, 1.0};
    const bool dv = amax != 1.0;
    parallel_spans(rows, K, nthreads, [&](int64_t r, int64_t a, int64_t b) {
        double *m = scratch(0, b - a + 2), *d = scratch(1, b - a + 1), *cr = scratch(2, (b - a) * 4);
        pchip_span(h.data(), K, y + r * K, a, b, m, d, cr);
        float *o = out + (r * (K - 1) + a) * 4;
        for (int64_t e = 0; e < (b - a) * 4; ++e) {
            double v = cr[e] * w[e & 3];
            if (dv) v = v / amax;
            o[e] = (float)v;
        }
    });
    return PSS_OK;
}

int pss_host_ppoly_eval(const double *x, int64_t K, const double *c, int64_t rows, const double *ph,
                        int64_t n, double *out, int nthreads) {
    if (K < 2 || rows < 0 || n < 0 || !x || !c || !ph || !out) return PSS_EINVAL;
    std::vector<int64_t> iv(n);
    std::vector<double> s(n);
    locate(x, K, ph, n, iv.data(), s.data());
    parallel_rows(rows, nthreads, [&](int64_t r0, int64_t r1) {
        for (int64_t r = r0; r < r1; ++r) {
            const double *cr = c + r * (K - 1) * 4;
            double *o = out + r * n;
            for (int64_t j = 0; j < n; ++j) o[j] = ppoly_at(cr + 4 * iv[j], s[j]);
        }
    });
    return PSS_OK;
}

int pss_host_device_table(const double *c, int64_t rows, int64_t nint, double h, double amax,
                          float *out, int nthreads) {
    if (rows < 0 || nint < 1 || !c || !out) return PSS_EINVAL;
    const double w[4] = {pow(h, 3.0), pow(h, 2.0), h, 1.0};   // np.array([h ** 3, h ** 2, h, 1.0])
    const bool div = amax != 1.0;
    parallel_rows(rows, nthreads, [&](int64_t r0, int64_t r1) {
        for (int64_t e = r0 * nint * 4; e < r1 * nint * 4; ++e) {
            double v = c[e] * w[e & 3];
            if (div) v = v / amax;
            out[e] = (float)v;
        }
    });
    return PSS_OK;
}

}  // extern "C"
