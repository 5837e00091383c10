// Native multi-threaded reader for the reference's matrix files:
// bigmemory::read.big.matrix(mat_file, type = 'double', sep = '\t')
// (R/TADpole.R:17, :160) -- a headerless tab-separated numeric matrix.
//
// The file is memory-mapped and cut into one byte range per thread at line
// boundaries; pass 1 counts the lines of every range (row offsets), pass 2
// parses each range's lines straight into the output (std::from_chars: the
// correctly rounded double of each field).  "NA", "NaN", "nan", "Inf" spellings
// and empty fields follow R's reader: NA/NaN/empty -> NaN (the pipeline maps
// them to 0 exactly as R/TADpole.R:19 does), Inf/-Inf -> +-infinity.  A
// line with fewer fields than the first line is padded with NaN; more fields
// is an error.  CRLF line ends are accepted.  Host code only (no device use).
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <charconv>
#include <condition_variable>
#include <mutex>
#include <cmath>
#include <cstring>
#include <string>
#include <functional>
#include <thread>
#include <vector>

#include "tp_internal.h"

namespace tp {

namespace {

struct Mapped {
    const char *p = nullptr;
    size_t n = 0;
    int fd = -1;
    explicit Mapped(const char *path) {
        fd = ::open(path, O_RDONLY);
        if (fd < 0) fail(TP_ERR_ARG, std::string("cannot open ") + path);
        struct stat st;
        if (fstat(fd, &st) != 0) fail(TP_ERR_ARG, std::string("cannot stat ") + path);
        n = (size_t)st.st_size;
        if (n > 0) {
            // no MAP_POPULATE: the reading threads fault their own ranges in parallel
            void *m = mmap(nullptr, n, PROT_READ, MAP_PRIVATE, fd, 0);
            if (m == MAP_FAILED) fail(TP_ERR_ARG, std::string("cannot map ") + path);
            p = (const char *)m;
            (void)madvise(m, n, MADV_SEQUENTIAL);
        }
    }
    ~Mapped() {
        if (p) munmap((void *)p, n);
        if (fd >= 0) ::close(fd);
    }
};

// end of the logical content (a final newline does not start an empty row)
size_t content_end(const Mapped &m) {
    size_t e = m.n;
    while (e > 0 && (m.p[e - 1] == '\n' || m.p[e - 1] == '\r')) --e;
    return e;
}

int count_fields(const char *b, const char *e) {
    if (b == e) return 0;
    int c = 1;
    for (const char *q = b; q < e; ++q) c += *q == '\t';
    return c;
}

double parse_field(const char *b, const char *e) {
    while (b < e && (*b == ' ' || *b == '"')) ++b;
    while (e > b && (e[-1] == ' ' || e[-1] == '\r' || e[-1] == '"')) --e;
    if (b == e) return std::nan("");
    const char *s = b;
    if (*s == '+') ++s;
    {   // fast path: plain integers (raw Hi-C counts), exact below 2^53
        const char *q = s;
        const bool neg = q < e && *q == '-';
        if (neg) ++q;
        if (q < e && e - q <= 15) {
            long long iv = 0;
            const char *z = q;
            while (z < e && (unsigned)(*z - '0') < 10u) iv = iv * 10 + (*z++ - '0');
            if (z == e) return neg ? -(double)iv : (double)iv;
        }
    }
    double v;
    auto r = std::from_chars(s, e, v);
    if (r.ec == std::errc() && r.ptr == e) return v;
    // R spellings from_chars does not take
    const size_t len = (size_t)(e - b);
    auto is = [&](const char *w) { return len == strlen(w) && strncasecmp(b, w, len) == 0; };
    if (is("Inf") || is("+Inf") || is("Infinity")) return HUGE_VAL;
    if (is("-Inf") || is("-Infinity")) return -HUGE_VAL;
    return std::nan("");   // NA, NaN and anything non-numeric (R: NA)
}

// [b, e) -> starts of lines inside it (the range starts at a line start)
size_t count_lines(const char *b, const char *e) {
    if (b >= e) return 0;
    size_t c = 0;
    const char *q = b;
    while (q < e) {
        const void *nl = memchr(q, '\n', (size_t)(e - q));
        ++c;
        if (!nl) break;
        q = (const char *)nl + 1;
    }
    return c;
}

}  // namespace

void tsv_dims(const char *path, int *nrow, int *ncol) {
    Mapped m(path);
    const size_t e = content_end(m);
    if (e == 0) {
        *nrow = 0;
        *ncol = 0;
        return;
    }
    const char *nl = (const char *)memchr(m.p, '\n', e);
    const char *le = nl ? nl : m.p + e;
    *ncol = count_fields(m.p, le);
    // line count: one byte range per hardware thread (a single memchr scan of
    // a 10k-bin file, 200 MB, was ~20 ms of TADpole(path))
    const int T = e < ((size_t)1 << 22) ? 1 : (int)std::max(1u, std::min(64u, std::thread::hardware_concurrency()));
    std::vector<size_t> cnt(T, 0);
    {
        std::vector<std::thread> th;
        for (int t = 0; t < T; ++t)
            th.emplace_back([&, t] {
                const char *b = m.p + e * (size_t)t / (size_t)T, *q = b, *end = m.p + e * (size_t)(t + 1) / (size_t)T;
                size_t c = 0;
                while (q < end) {
                    const void *x = memchr(q, '\n', (size_t)(end - q));
                    if (!x) break;
                    ++c;
                    q = (const char *)x + 1;
                }
                cnt[t] = c;
            });
        for (auto &x : th) x.join();
    }
    size_t rows = 1;   // newlines inside the content + the last line (no trailing newline counted)
    for (size_t c : cnt) rows += c;
    if (rows > 0x7fffffff) fail(TP_ERR_UNSUPPORTED, "too many rows");
    *nrow = (int)rows;
}

void tsv_read(const char *path, int nrow, int ncol, int nthreads, bool row_major, double *out) {
    Mapped m(path);
    const size_t e = content_end(m);
    if (nrow == 0 || ncol == 0) return;
    int T = std::max(1, std::min(nthreads, 64));
    if (e < (size_t)T * 65536) T = 1;
    // chunk boundaries at line starts
    std::vector<size_t> start(T + 1);
    start[0] = 0;
    start[T] = e;
    for (int t = 1; t < T; ++t) {
        size_t s = e * (size_t)t / (size_t)T;
        if (s < start[t - 1]) s = start[t - 1];
        const void *nl = s < e ? memchr(m.p + s, '\n', e - s) : nullptr;
        start[t] = nl ? (size_t)((const char *)nl - m.p) + 1 : e;
    }
    std::vector<size_t> rows(T, 0);
    {
        std::vector<std::thread> th;
        for (int t = 0; t < T; ++t)
            th.emplace_back([&, t] { rows[t] = count_lines(m.p + start[t], m.p + start[t + 1]); });
        for (auto &x : th) x.join();
    }
    std::vector<size_t> row0(T + 1, 0);
    for (int t = 0; t < T; ++t) row0[t + 1] = row0[t] + rows[t];
    if (row0[T] != (size_t)nrow) fail(TP_ERR_ARG, "row count changed while reading (or wrong nrow)");
    std::vector<long> bad_line(T, -1);
    // row-major parse target: `out` itself, or a scratch buffer transposed afterwards
    std::vector<double> scratch;
    double *dst = out;
    if (!row_major) {
        scratch.resize((size_t)nrow * ncol);
        dst = scratch.data();
    }
    {
        std::vector<std::thread> th;
        for (int t = 0; t < T; ++t)
            th.emplace_back([&, t] {
                const char *q = m.p + start[t], *end = m.p + start[t + 1];
                size_t r = row0[t];
                while (q < end) {
                    const char *nl = (const char *)memchr(q, '\n', (size_t)(end - q));
                    const char *le = nl ? nl : end;
                    double *row = dst + r * (size_t)ncol;
                    int c = 0;
                    const char *f = q;
                    while (true) {
                        const char *tab = (const char *)memchr(f, '\t', (size_t)(le - f));
                        const char *fe = tab ? tab : le;
                        if (c >= ncol) {
                            if (bad_line[t] < 0) bad_line[t] = (long)r;
                            break;
                        }
                        row[c++] = parse_field(f, fe);
                        if (!tab) break;
                        f = tab + 1;
                    }
                    for (; c < ncol; ++c) row[c] = std::nan("");
                    ++r;
                    q = nl ? nl + 1 : end;
                }
            });
        for (auto &x : th) x.join();
    }
    for (int t = 0; t < T; ++t)
        if (bad_line[t] >= 0)
            fail(TP_ERR_ARG, "line " + std::to_string(bad_line[t] + 1) + " has more than " + std::to_string(ncol) +
                                 " fields");
    if (!row_major) {   // blocked transpose into the column-major output
        const int BT = 64;
        std::vector<std::thread> th;
        for (int t = 0; t < T; ++t)
            th.emplace_back([&, t] {
                for (int i0 = t * BT; i0 < nrow; i0 += T * BT)
                    for (int j0 = 0; j0 < ncol; j0 += BT)
                        for (int i = i0; i < std::min(nrow, i0 + BT); ++i)
                            for (int j = j0; j < std::min(ncol, j0 + BT); ++j)
                                out[(size_t)j * nrow + i] = scratch[(size_t)i * ncol + j];
            });
        for (auto &x : th) x.join();
    }
}

// Row-major parse in row blocks of about block_bytes of text each, through a
// ring of `nslots` staging slots: alloc(slot_rows) returns nslots x slot_rows
// x ncol doubles (called once, after the line count); block b is parsed into
// slot b % nslots (row r at (r - r0) * ncol), and on_block(r0, r1, rows, slot)
// runs on the calling thread as soon as it is complete, while the worker
// threads parse the next blocks (thread t takes byte range t of every block,
// block after block).  A slot is written again only after slot_free(slot)
// returned on the calling thread (the caller waits there for its upload of
// the slot), so the staging is nslots blocks, not the matrix.  Errors (a line
// with too many fields) are raised after the last block.
void tsv_read_rows(const char *path, int nrow, int ncol, int nthreads, size_t block_bytes, int nslots,
                   const std::function<double *(size_t)> &alloc,
                   const std::function<void(size_t, size_t, const double *, int)> &on_block,
                   const std::function<void(int)> &slot_free) {
    Mapped m(path);
    const size_t e = content_end(m);
    if (nrow == 0 || ncol == 0) return;
    int T = std::max(1, std::min(nthreads, 64));
    const int S = std::max(2, nslots);
    const size_t dbytes = (size_t)nrow * (size_t)ncol * sizeof(double);
    int NB = (int)std::min<size_t>(4096, std::max<size_t>(2 * (size_t)S, dbytes / std::max<size_t>(block_bytes, 65536) + 1));
    if (e < (size_t)T * NB * 65536) T = 1;
    if (e < (size_t)NB * 65536) NB = std::max<int>(1, (int)(e / 65536));
    const int Q = NB * T;
    std::vector<size_t> start(Q + 1);
    start[0] = 0;
    start[Q] = e;
    for (int q = 1; q < Q; ++q) {
        size_t s = e * (size_t)q / (size_t)Q;
        if (s < start[q - 1]) s = start[q - 1];
        const void *nl = s < e ? memchr(m.p + s, '\n', e - s) : nullptr;
        start[q] = nl ? (size_t)((const char *)nl - m.p) + 1 : e;
    }
    std::vector<size_t> rows(Q, 0);
    {
        std::vector<std::thread> th;
        for (int t = 0; t < T; ++t)
            th.emplace_back([&, t] {
                for (int q = t; q < Q; q += T) rows[q] = count_lines(m.p + start[q], m.p + start[q + 1]);
            });
        for (auto &x : th) x.join();
    }
    std::vector<size_t> row0(Q + 1, 0);
    for (int q = 0; q < Q; ++q) row0[q + 1] = row0[q] + rows[q];
    if (row0[Q] != (size_t)nrow) fail(TP_ERR_ARG, "row count changed while reading (or wrong nrow)");
    size_t slot_rows = 1;
    for (int b = 0; b < NB; ++b) slot_rows = std::max(slot_rows, row0[(size_t)(b + 1) * T] - row0[(size_t)b * T]);
    double *ring = alloc(slot_rows);
    std::vector<long> bad_line(T, -1);
    // blocking hand-offs (no spinning: on a CPU-quota'd host, spinning
    // waiters steal the parse's time slices): workers wait for their block's
    // slot, the calling thread for each block's completion
    std::mutex mu;
    std::condition_variable cv_work, cv_main;
    std::vector<int> done(NB, 0);
    int writable = std::min(NB, S);   // blocks [0, writable) may be written
    bool stop = false;
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t)
        th.emplace_back([&, t] {
            for (int b = 0; b < NB; ++b) {
                {
                    std::unique_lock<std::mutex> lk(mu);
                    cv_work.wait(lk, [&] { return stop || b < writable; });
                    if (b >= writable) return;
                }
                const int q = b * T + t;
                const char *p = m.p + start[q], *end = m.p + start[q + 1];
                size_t r = row0[q];
                const size_t rb0 = row0[(size_t)b * T];
                double *slot = ring + (size_t)(b % S) * slot_rows * (size_t)ncol;
                while (p < end) {
                    const char *nl = (const char *)memchr(p, '\n', (size_t)(end - p));
                    const char *le = nl ? nl : end;
                    double *row = slot + (r - rb0) * (size_t)ncol;
                    int c = 0;
                    const char *f = p;
                    while (true) {
                        const char *tab = (const char *)memchr(f, '\t', (size_t)(le - f));
                        const char *fe = tab ? tab : le;
                        if (c >= ncol) {
                            if (bad_line[t] < 0) bad_line[t] = (long)r;
                            break;
                        }
                        row[c++] = parse_field(f, fe);
                        if (!tab) break;
                        f = tab + 1;
                    }
                    for (; c < ncol; ++c) row[c] = std::nan("");
                    ++r;
                    p = nl ? nl + 1 : end;
                }
                bool last;
                {
                    std::lock_guard<std::mutex> lk(mu);
                    last = ++done[b] == T;
                }
                if (last) cv_main.notify_one();
            }
        });
    struct Join {   // the workers finish even when on_block / slot_free throws
        std::vector<std::thread> &th;
        std::mutex &mu;
        std::condition_variable &cv;
        bool &stop;
        ~Join() {
            {
                std::lock_guard<std::mutex> lk(mu);
                stop = true;
            }
            cv.notify_all();
            for (auto &x : th)
                if (x.joinable()) x.join();
        }
    } join{th, mu, cv_work, stop};
    for (int b = 0; b < NB; ++b) {
        {
            std::unique_lock<std::mutex> lk(mu);
            cv_main.wait(lk, [&] { return done[b] == T; });
        }
        on_block(row0[(size_t)b * T], row0[(size_t)(b + 1) * T], ring + (size_t)(b % S) * slot_rows * (size_t)ncol,
                 b % S);
        if (b + S < NB) {   // block b + S reuses this slot once its upload is done
            slot_free(b % S);
            {
                std::lock_guard<std::mutex> lk(mu);
                writable = b + S + 1;
            }
            cv_work.notify_all();
        }
    }
    for (auto &x : th) x.join();
    for (int t = 0; t < T; ++t)
        if (bad_line[t] >= 0)
            fail(TP_ERR_ARG, "line " + std::to_string(bad_line[t] + 1) + " has more than " + std::to_string(ncol) +
                                 " fields");
}

}  // namespace tp
