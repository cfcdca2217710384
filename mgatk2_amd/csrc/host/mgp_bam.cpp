// mgp_bam.cpp — BAM ingest for the MI355X pileup engine (host side, libmgphost.so).
//
// Replaces pysam under BAMReader (src/processing/readers.py:35-165): BGZF
// inflate on a thread pool, `.bai` seek to the first chrM record (what
// `bam.fetch(mito_chr)` does, readers.py:87-88), record decode and packing into
// the engine's SoA batch + payload records (include/mgpileup.h), CB-tag
// whitelist lookup (readers.py:104-111). Also the tag count of the barcode
// auto-extraction pass (src/file_io/barcode_extraction.py:22-32).
#include <zlib.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <functional>
#include <mutex>
#include <cerrno>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <new>
#include <fcntl.h>
#include <string>
#include <thread>
#include <unistd.h>
#include <unordered_map>
#include <utility>
#include <vector>

#include "../../../include/mgpileup.h"
#include "../../../include/mgpileup_host.h"
#include "mgp_pack32_host.h"
#include "mgp_pool.h"
#include "mgp_zcodec.h"
#include "mgp_place.h"

// one thread-local error string for every entry point of libmgphost.so
std::string& mgp_host_err() {
    static thread_local std::string e;
    return e;
}

namespace {

// MGP_HOST_PROFILE=1: phase times of mgp_bam_read_ref on stderr
double now_s() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
thread_local double t_inflate = 0, t_pread = 0;

#define g_err mgp_host_err()
int fail(const std::string& m) {
    g_err = m;
    return -1;
}

inline uint16_t rd16(const uint8_t* p) { uint16_t v; std::memcpy(&v, p, 2); return v; }
inline uint32_t rd32(const uint8_t* p) { uint32_t v; std::memcpy(&v, p, 4); return v; }
inline int32_t rdi32(const uint8_t* p) { int32_t v; std::memcpy(&v, p, 4); return v; }
inline uint64_t rd64(const uint8_t* p) { uint64_t v; std::memcpy(&v, p, 8); return v; }

// barcode hash: 8 bytes per step (a per-byte FNV loop was most of a lookup's time)
inline uint64_t hash_bytes(const char* s, size_t n) {
    uint64_t h = 0x9E3779B97F4A7C15ull ^ (uint64_t)n;
    size_t i = 0;
    for (; i + 8 <= n; i += 8) {
        uint64_t w;
        std::memcpy(&w, s + i, 8);
        h = (h ^ w) * 0xBF58476D1CE4E5B9ull;
        h ^= h >> 31;
    }
    if (i < n) {
        uint64_t w = 0;
        std::memcpy(&w, s + i, n - i);
        h = (h ^ w) * 0x94D049BB133111EBull;
        h ^= h >> 29;
    }
    return h;
}

// open-addressing string -> index table (no allocation per lookup): the keys' bytes
// in one pool, each slot's hash, key offset, length and value side by side
struct StrTable {
    struct Slot {
        uint64_t hash;
        uint32_t off, len;
        int32_t val, used;
    };
    std::vector<char> pool;
    std::vector<Slot> slots;
    std::vector<int32_t> vals;  // the values (for n_keys)
    uint64_t mask = 0;
    void build(const std::vector<std::string>& k, const std::vector<int32_t>& v) {
        size_t cap = 16;
        while (cap < k.size() * 2 + 1) cap <<= 1;
        slots.assign(cap, Slot{0, 0, 0, -1, 0});
        mask = cap - 1;
        pool.clear();
        vals.clear();
        for (size_t i = 0; i < k.size(); ++i) put(k[i], v[i]);
    }
    void put(const std::string& key, int32_t v) {
        const uint64_t h = hash_bytes(key.data(), key.size());
        uint64_t s = h & mask;
        while (slots[s].used) {
            Slot& x = slots[s];
            if (x.hash == h && x.len == key.size() && std::memcmp(pool.data() + x.off, key.data(), key.size()) == 0) {
                x.val = v;  // last duplicate wins (dict semantics)
                vals.push_back(v);
                return;
            }
            s = (s + 1) & mask;
        }
        slots[s] = Slot{h, (uint32_t)pool.size(), (uint32_t)key.size(), v, 1};
        pool.insert(pool.end(), key.begin(), key.end());
        vals.push_back(v);
    }
    int32_t get(const char* p, size_t n) const {
        if (slots.empty()) return -1;
        const uint64_t h = hash_bytes(p, n);
        uint64_t s = h & mask;
        while (slots[s].used) {
            const Slot& x = slots[s];
            if (x.hash == h && x.len == n && std::memcmp(pool.data() + x.off, p, n) == 0) return x.val;
            s = (s + 1) & mask;
        }
        return -1;
    }
};

struct Block {
    uint64_t coff;     // compressed offset of the block
    uint32_t csize;    // whole block size
    uint32_t isize;    // inflated size
    size_t out_off;    // offset in the inflated buffer
};

}  // namespace

struct mgp_bam {
    int fd = -1;
    std::string path;
    int n_threads = 1;
    int64_t file_size = 0;
    std::vector<std::string> ref_names;
    std::vector<int64_t> ref_lens;
    uint64_t first_record_voff = 0;  // virtual offset right after the header
    bool has_index = false;
    std::vector<uint64_t> ref_first_voff;  // from the index; UINT64_MAX if the ref has no reads
    std::vector<int64_t> ref_records;      // mapped + placed unmapped records (index pseudo-bin), -1 unknown
    StrTable wl;
    char tag[2] = {'C', 'B'};
    int32_t bulk_cell = -1;  // >= 0: every record goes to this cell (bulk calling)
    bool pack = false;       // write the packed record layout where a read fits
    bool pack32 = false;     // ... the 32-byte layout first, made for pack32_minq (mgp_bam_set_pack32)
    int pack32_minq = 0;
    int pack32_dist = 5;
    int placement = MGP_PLACE_DENSE;  // payload placement (mgp_place_records)
};

namespace {

// Reads [off, off+n) of the file.
bool pread_all(int fd, uint8_t* dst, size_t n, uint64_t off) {
    size_t done = 0;
    while (done < n) {
        ssize_t r = ::pread(fd, dst + done, n - done, (off_t)(off + done));
        if (r < 0) {
            if (errno == EINTR) continue;
            return false;
        }
        if (r == 0) return false;
        done += (size_t)r;
    }
    return true;
}

// Parse the BGZF block header at p (n bytes available); returns the block size or 0.
uint32_t bgzf_block_size(const uint8_t* p, size_t n) {
    if (n < 18 || p[0] != 31 || p[1] != 139 || p[2] != 8 || !(p[3] & 4)) return 0;
    const uint16_t xlen = rd16(p + 10);
    if (n < (size_t)12 + xlen) return 0;
    const uint8_t* x = p + 12;
    size_t i = 0;
    while (i + 4 <= xlen) {
        const uint16_t slen = rd16(x + i + 2);
        if (x[i] == 66 && x[i + 1] == 67 && slen == 2) return (uint32_t)rd16(x + i + 4) + 1;
        i += 4 + slen;
    }
    return 0;
}

bool inflate_block(const uint8_t* blk, uint32_t csize, uint8_t* out, uint32_t isize, mgp_host::Inflator& inf) {
    const uint16_t xlen = rd16(blk + 10);
    const uint8_t* cdata = blk + 12 + xlen;
    const uint32_t clen = csize - 12 - xlen - 8;
    if (!inf.raw(cdata, clen, out, isize)) return false;
    const uint32_t crc = rd32(blk + csize - 8);
    return mgp_host::crc32_any(0, out, isize) == crc;
}

// A thread that runs one job at a time (the stream decode's serial placement, beside
// the pool's passes over the next chunk; the prefetch's boundary walk, beside the
// next chunk's read and inflate).
class Worker {
  public:
    Worker() : th_([this] { loop(); }) {}
    ~Worker() {
        {
            std::lock_guard<std::mutex> g(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        th_.join();
    }
    void submit(std::function<void()> f) {
        std::lock_guard<std::mutex> g(mu_);
        job_ = std::move(f);
        busy_ = true;
        cv_.notify_all();
    }
    void wait() {
        std::unique_lock<std::mutex> g(mu_);
        cv_.wait(g, [&] { return !busy_; });
    }

  private:
    void loop() {
        std::unique_lock<std::mutex> g(mu_);
        for (;;) {
            cv_.wait(g, [&] { return stop_ || (busy_ && job_); });
            if (stop_) return;
            std::function<void()> f = std::move(job_);
            job_ = nullptr;
            g.unlock();
            f();
            g.lock();
            busy_ = false;
            cv_.notify_all();
        }
    }
    std::mutex mu_;
    std::condition_variable cv_;
    std::function<void()> job_;
    bool busy_ = false, stop_ = false;
    std::thread th_;
};

// An inflated chunk of the BGZF stream: the bytes of consecutive whole blocks at
// mem + kHead (the room in front takes the partial record the consumer carries over
// from the chunk before).
constexpr size_t kHead = 1u << 20;
struct Chunk {
    std::unique_ptr<uint8_t[]> mem;
    size_t cap = 0;
    size_t n = 0;       // inflated bytes at mem + kHead
    bool last = false;  // the end of the file follows
    // the records that start in this chunk (offsets from mem + kHead), their block sizes
    // and reference ids, when the prefetch thread walked them (walked)
    bool walked = false;
    std::vector<uint32_t> rstart, rsize;
    std::vector<int32_t> rref;
};

// Reads and inflates the BGZF stream ahead of the consumer on a thread of its own
// (its blocks inflated on a pool of the bam's threads), so the file reads and the
// inflate overlap the decode of the chunk before. Chunks start at 64 KiB of
// compressed bytes (a header or a tag check needs little) and grow x4 up to 16 MiB;
// at most two wait for the consumer.
class Prefetch {
  public:
    // walk_from >= 0: the prefetch thread also walks the record boundaries of every chunk,
    // the first record starting walk_from bytes into the first chunk (the stream decode's
    // serial boundary walk, off the consumer's thread)
    Prefetch(mgp_bam* bam, uint64_t coff, int64_t walk_from = -1)
        : bam_(bam), coff_(coff), pool_(std::max(1, bam->n_threads)), walking_(walk_from >= 0),
          wnext_(walk_from) {
        th_ = std::thread([this] { run(); });
    }
    ~Prefetch() {
        join();
        for (Chunk* c : ready_) delete c;
        for (Chunk* c : free_) delete c;
    }
    // stops the prefetch thread and waits for it (its profile counters are then stable)
    void join() {
        {
            std::lock_guard<std::mutex> g(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        if (th_.joinable()) th_.join();
    }
    // the next chunk in file order; nullptr on error (message in err())
    Chunk* next() {
        std::unique_lock<std::mutex> g(mu_);
        cv_.wait(g, [&] { return !ready_.empty() || failed_; });
        if (ready_.empty()) return nullptr;
        Chunk* c = ready_.front();
        ready_.pop_front();
        cv_.notify_all();
        return c;
    }
    void recycle(Chunk* c) {
        {
            std::lock_guard<std::mutex> g(mu_);
            free_.push_back(c);
        }
        cv_.notify_all();
    }
    const std::string& err() const { return err_; }
    double t_pread = 0, t_inflate = 0, t_walk = 0;

  private:
    static constexpr size_t kMaxBatch = 16u << 20;
    static constexpr size_t kAhead = 2;
    void set_fail(const std::string& m) {
        std::lock_guard<std::mutex> g(mu_);
        err_ = m;
        failed_ = true;
        cv_.notify_all();
    }
    // record boundaries of chunk c, continuing the chain from the chunk before: wnext_ =
    // where the next record starts in this chunk, or (negative, -k) a record whose 4-byte
    // size field has its first k bytes (wpart_) at the end of the chunk before. A size
    // below 32 stops the walk (the consumer then walks itself and reports the record).
    void walk(Chunk* c) {
        c->walked = false;
        c->rstart.clear();
        c->rsize.clear();
        c->rref.clear();
        if (!walking_) return;
        const uint8_t* d = c->mem.get() + kHead;
        const size_t n = c->n;
        int64_t q = wnext_;
        if (q < 0) {
            const size_t k = (size_t)(-q);
            if (n < 4 - k) {  // (a chunk of fewer bytes than the field's rest: not walked)
                walking_ = false;
                return;
            }
            uint8_t f[4];
            std::memcpy(f, wpart_, k);
            std::memcpy(f + k, d, 4 - k);
            q = (int64_t)(4 + rd32(f)) - (int64_t)k;
        }
        while ((uint64_t)q + 4 <= n) {
            const uint32_t bs = rd32(d + q);
            if (bs < 32) {
                walking_ = false;
                return;
            }
            c->rstart.push_back((uint32_t)q);
            c->rsize.push_back(bs);
            c->rref.push_back((uint64_t)q + 8 <= n ? rdi32(d + q + 4) : INT32_MIN);  // (split: the consumer reads it)
            q += 4 + (int64_t)bs;
        }
        if ((uint64_t)q < n) {
            const size_t k = n - (size_t)q;
            std::memcpy(wpart_, d + q, k);
            wnext_ = -(int64_t)k;
        } else {
            wnext_ = q - (int64_t)n;
        }
        c->walked = true;
    }
    void run() {
        struct Settle {
            Prefetch* p;
            ~Settle() { p->settle_walk(); }
        } settle{this};
        size_t want_c = 64u << 10;
        std::vector<uint8_t> raw;
        std::vector<Block> blocks;
        bool last = false;
        while (!last) {
            Chunk* c = nullptr;
            {
                std::unique_lock<std::mutex> g(mu_);
                cv_.wait(g, [&] { return stop_ || ready_.size() < kAhead; });
                if (stop_) return;
                if (!free_.empty()) {
                    c = free_.back();
                    free_.pop_back();
                }
            }
            if (!c) c = new (std::nothrow) Chunk();
            if (!c) return set_fail("out of host memory");
            c->n = 0;
            c->last = false;
            c->walked = false;
            if (coff_ >= (uint64_t)bam_->file_size) {
                c->last = last = true;
            } else {
                size_t want = (size_t)std::min<uint64_t>(want_c, (uint64_t)bam_->file_size - coff_);
                want_c = std::min(kMaxBatch, want_c * 4);
                // whole blocks only; a block larger than the read: read it alone
                for (;;) {
                    const double tr0 = now_s();
                    bool rd_ok;
                    if (ahead_want_ && ahead_coff_ == coff_ && ahead_want_ == want) {  // read during the last inflate
                        reader_.wait();
                        raw.swap(ahead_);
                        rd_ok = ahead_ok_;
                    } else {
                        if (ahead_want_) reader_.wait();
                        raw.resize(want);
                        rd_ok = pread_all(bam_->fd, raw.data(), want, coff_);
                    }
                    ahead_want_ = 0;
                    t_pread += now_s() - tr0;
                    if (!rd_ok) return delete c, set_fail("read error in " + bam_->path);
                    blocks.clear();
                    size_t p = 0, total = 0;
                    while (p < want) {
                        const uint32_t bs = bgzf_block_size(raw.data() + p, want - p);
                        if (bs == 0) {
                            if (blocks.empty() && want - p >= 18)
                                return delete c, set_fail("not a BGZF block at offset " + std::to_string(coff_ + p));
                            break;
                        }
                        if (p + bs > want) break;  // partial block: next chunk
                        Block b;
                        b.coff = p;
                        b.csize = bs;
                        b.isize = rd32(raw.data() + p + bs - 4);
                        if (b.isize > 65536 || bs < 12u + rd16(raw.data() + p + 10) + 8u)
                            return delete c, set_fail("corrupt BGZF block at offset " + std::to_string(coff_ + p));
                        b.out_off = total;
                        total += b.isize;
                        blocks.push_back(b);
                        p += bs;
                    }
                    if (!blocks.empty()) {
                        // (MGP_BAM_READ_AHEAD=1: the next chunk's compressed bytes read on the
                        // reader while this one inflates)
                        if (read_ahead_ && coff_ + p < (uint64_t)bam_->file_size) {
                            ahead_coff_ = coff_ + p;
                            ahead_want_ = (size_t)std::min<uint64_t>(want_c, (uint64_t)bam_->file_size - ahead_coff_);
                            reader_.submit([this] {
                                ahead_.resize(ahead_want_);
                                ahead_ok_ = pread_all(bam_->fd, ahead_.data(), ahead_want_, ahead_coff_);
                            });
                        }
                        if (kHead + total > c->cap) {
                            c->cap = kHead + total + (total >> 3);
                            c->mem.reset(new (std::nothrow) uint8_t[c->cap]);
                            if (!c->mem) return delete c, set_fail("out of host memory");
                        }
                        std::atomic<size_t> next{0};
                        std::atomic<bool> ok{true};
                        const int nt = std::max(1, std::min<int>(pool_.size(), (int)blocks.size()));
                        uint8_t* out = c->mem.get() + kHead;
                        const double ti0 = now_s();
                        pool_.run(nt, [&](int) {
                            mgp_host::Inflator inf;
                            for (;;) {
                                const size_t i = next.fetch_add(1);
                                if (i >= blocks.size()) break;
                                const Block& b = blocks[i];
                                if (!inflate_block(raw.data() + b.coff, b.csize, out + b.out_off, b.isize, inf)) {
                                    ok = false;
                                    break;
                                }
                            }
                        });
                        t_inflate += now_s() - ti0;
                        if (!ok) return delete c, set_fail("BGZF inflate/CRC error in " + bam_->path);
                        c->n = total;
                        coff_ += p;
                        c->last = last = coff_ >= (uint64_t)bam_->file_size;
                        break;
                    }
                    // no whole block in `want` bytes: the block at coff_ alone
                    if (want < 18) return delete c, set_fail("truncated BGZF");
                    const uint32_t bs = bgzf_block_size(raw.data(), want);
                    if (!bs) return delete c, set_fail("bad BGZF header");
                    if (coff_ + bs > (uint64_t)bam_->file_size)
                        return delete c, set_fail("truncated BGZF block at offset " + std::to_string(coff_) + " in " +
                                                  bam_->path);
                    want = bs;
                }
            }
            // the chunk before leaves its walk first (chunks reach the consumer in file
            // order); this one's walk then runs on the walker while the loop reads and
            // inflates the next (the walk is a serial chain: ~30 % of this thread's time)
            walker_.wait();
            if (walked_) push_ready(std::exchange(walked_, nullptr));
            if (walk_async_ && walking_ && c->n > 0 && !last) {
                walked_ = c;
                walker_.submit([this, c] {
                    const double tw0 = now_s();
                    walk(c);
                    t_walk += now_s() - tw0;
                });
            } else {
                const double tw0 = now_s();
                walk(c);
                t_walk += now_s() - tw0;
                push_ready(c);
            }
        }
    }
    void push_ready(Chunk* c) {
        {
            std::lock_guard<std::mutex> g(mu_);
            ready_.push_back(c);
        }
        cv_.notify_all();
    }
    // (every return of run(): a chunk still on the walker goes to ready_, which the
    // destructor frees)
    void settle_walk() {
        reader_.wait();
        walker_.wait();
        if (walked_) push_ready(std::exchange(walked_, nullptr));
    }
    mgp_bam* bam_;
    uint64_t coff_;
    mgp_host::Pool pool_;  // (before th_: alive while run() uses it)
    Worker walker_;        // (likewise)
    Worker reader_;        // (likewise; its read targets ahead_)
    std::vector<uint8_t> ahead_;
    uint64_t ahead_coff_ = 0;
    size_t ahead_want_ = 0;  // 0: no read ahead pending
    bool ahead_ok_ = false;
    // (MGP_BAM_READ_AHEAD=1: the next chunk read during this one's inflate. Off: on the
    // box's 16-core share the kernel's copy competes with the inflate pool, C4 ingest
    // 3.71-3.95 s against 3.68-3.73 s reading in line, profiles/r05/e2e_walk_r5u_*.log)
    const bool read_ahead_ = [] {
        const char* e = std::getenv("MGP_BAM_READ_AHEAD");
        return e && std::strtol(e, nullptr, 10) != 0;
    }();
    Chunk* walked_ = nullptr;  // the chunk on the walker
    // (MGP_BAM_WALK_ASYNC=0: the walk on this thread, between inflates; C4 ingest 4.80-5.21 s
    // against 3.65-4.00 s with the walker, profiles/r05/e2e_walk_r5t_*.log)
    const bool walk_async_ = [] {
        const char* e = std::getenv("MGP_BAM_WALK_ASYNC");
        return !e || std::strtol(e, nullptr, 10) != 0;
    }();
    bool walking_;
    int64_t wnext_;
    uint8_t wpart_[4] = {0, 0, 0, 0};
    std::thread th_;
    std::mutex mu_;
    std::condition_variable cv_;
    std::deque<Chunk*> ready_;
    std::vector<Chunk*> free_;
    bool stop_ = false, failed_ = false;
    std::string err_;
};

// A sequential reader over the inflated BGZF stream: the consumer's view of the
// prefetched chunks ([base + pos, base + size) is valid until the next fill).
struct Stream {
    mgp_bam* bam = nullptr;
    std::unique_ptr<Prefetch> pf;
    Chunk* cur = nullptr;
    std::vector<uint8_t> big;  // a carried record larger than kHead, with the chunk after it
    const uint8_t* base = nullptr;
    size_t size = 0, pos = 0;
    bool eof = false;
    // hold: buffers left behind by advance() stay allocated until release_held() (the
    // pipelined stream decode still reads records of the chunk before)
    bool hold = false;
    std::vector<Chunk*> held;
    std::vector<std::vector<uint8_t>> held_big;
    // the record boundaries of [base, base + size) from the prefetch thread's walk
    // (walked): the carried record at 0 when wt > 0, then the chunk's records at wt +
    // wc->rstart[i] (block sizes wc->rsize, reference ids wc->rref)
    bool walked = false;
    const Chunk* wc = nullptr;
    size_t wt = 0;

    ~Stream() {
        release_held();
        if (cur && pf) pf->recycle(cur);
        if (pf) {  // (the profile counters of mgp_bam_read_ref, read once the prefetch thread has ended)
            pf->join();
            t_pread += pf->t_pread;
            t_inflate += pf->t_inflate;
        }
        pf.reset();
    }
    void release_held() {
        for (Chunk* c : held)
            if (pf) pf->recycle(c);
            else delete c;
        held.clear();
        held_big.clear();
    }
    bool fill(size_t need) {
        while (size - pos < need && !eof)
            if (!advance()) return false;
        return size - pos >= need;
    }
    bool advance() {
        Chunk* nx = pf->next();
        if (!nx) return fail(pf->err()), false;
        if (nx->n == 0) {  // (the end of the file: nothing to append)
            eof = nx->last;
            pf->recycle(nx);
            return true;
        }
        const size_t t = size - pos;  // the partial record carried over
        if (t <= kHead) {
            uint8_t* dst = nx->mem.get() + kHead - t;
            if (t) std::memcpy(dst, base + pos, t);
            base = dst;
        } else {
            std::vector<uint8_t> nb(t + nx->n);
            std::memcpy(nb.data(), base + pos, t);
            std::memcpy(nb.data() + t, nx->mem.get() + kHead, nx->n);
            big.swap(nb);
            base = big.data();
            if (hold && !nb.empty()) held_big.push_back(std::move(nb));
        }
        size = t + nx->n;
        pos = 0;
        eof = nx->last;
        // the buffer's boundaries: the carried record at 0, then the chunk's walked records
        walked = nx->walked && size >= 8;
        wc = nx;
        wt = t;
        if (cur) {
            if (hold) held.push_back(cur);
            else pf->recycle(cur);
        }
        cur = nx;
        return true;
    }
    const uint8_t* peek() const { return base + pos; }
    size_t avail() const { return size - pos; }
};

// walk: the prefetch thread also walks the record boundaries from voff on (Stream::walked)
bool stream_at(mgp_bam* bam, uint64_t voff, Stream& st, bool walk = false) {
    st.bam = bam;
    st.pf.reset();
    st.cur = nullptr;
    st.base = nullptr;
    st.size = st.pos = 0;
    st.eof = false;
    st.walked = false;
    st.pf.reset(new Prefetch(bam, voff >> 16, walk ? (int64_t)(voff & 0xFFFF) : -1));
    const size_t uoff = voff & 0xFFFF;
    if (uoff) {
        if (!st.fill(uoff)) return false;
        st.pos += uoff;
    }
    return true;
}

int parse_header(mgp_bam* bam) {
    Stream st;
    if (!stream_at(bam, 0, st)) return -1;
    if (!st.fill(12)) return fail(g_err.empty() ? "truncated BAM header" : g_err);
    const uint8_t* p = st.peek();
    if (std::memcmp(p, "BAM\1", 4) != 0) return fail("not a BAM file (bad magic)");
    const uint32_t l_text = rd32(p + 4);
    if (!st.fill(8 + (size_t)l_text + 4)) return fail("truncated BAM header text");
    st.pos += 8 + l_text;
    const int32_t n_ref = rdi32(st.peek());
    st.pos += 4;
    if (n_ref < 0) return fail("negative n_ref");
    // header bytes: magic + l_text + text + n_ref + sum(l_name + name + l_ref)
    uint64_t hlen = 12 + (uint64_t)l_text;
    for (int32_t r = 0; r < n_ref; ++r) {
        if (!st.fill(4)) return fail("truncated reference list");
        const uint32_t l_name = rd32(st.peek());
        if (!st.fill(4 + (size_t)l_name + 4)) return fail("truncated reference entry");
        const char* nm = (const char*)st.peek() + 4;
        bam->ref_names.emplace_back(nm, strnlen(nm, l_name));
        bam->ref_lens.push_back(rdi32(st.peek() + 4 + l_name));
        st.pos += 4 + l_name + 4;
        hlen += 4 + (uint64_t)l_name + 4;
    }
    // virtual offset of the first record: walk the blocks to the header's end
    uint64_t coff = 0, acc = 0;
    for (;;) {
        uint8_t h[18];
        if (!pread_all(bam->fd, h, 18, coff)) return fail("truncated BGZF while locating records");
        const uint32_t bs = bgzf_block_size(h, 18);
        if (!bs) return fail("bad BGZF block while locating records");
        uint8_t tail[4];
        if (!pread_all(bam->fd, tail, 4, coff + bs - 4)) return fail("truncated BGZF block");
        const uint32_t isz = rd32(tail);
        if (acc + isz > hlen) {
            bam->first_record_voff = (coff << 16) | (hlen - acc);
            break;
        }
        acc += isz;
        coff += bs;
        if (acc == hlen) {
            bam->first_record_voff = coff << 16;
            break;
        }
    }
    return 0;
}

int load_index(mgp_bam* bam) {
    const std::string ipath = bam->path + ".bai";
    FILE* f = std::fopen(ipath.c_str(), "rb");
    if (!f) return 0;
    std::vector<uint8_t> d;
    {
        std::fseek(f, 0, SEEK_END);
        const long sz = std::ftell(f);
        std::fseek(f, 0, SEEK_SET);
        d.resize((size_t)std::max(0L, sz));
        if (sz > 0 && std::fread(d.data(), 1, d.size(), f) != d.size()) {
            std::fclose(f);
            return fail("cannot read " + ipath);
        }
        std::fclose(f);
    }
    size_t p = 0;
    auto need = [&](size_t n) { return p + n <= d.size(); };
    if (!need(8) || std::memcmp(d.data(), "BAI\1", 4) != 0) return fail("bad BAI magic in " + ipath);
    const int32_t n_ref = rdi32(d.data() + 4);
    p = 8;
    if (n_ref != (int32_t)bam->ref_names.size()) return fail("BAI reference count does not match the BAM");
    bam->ref_first_voff.assign((size_t)n_ref, UINT64_MAX);
    bam->ref_records.assign((size_t)n_ref, -1);
    for (int32_t r = 0; r < n_ref; ++r) {
        if (!need(4)) return fail("truncated BAI");
        const int32_t n_bin = rdi32(d.data() + p);
        p += 4;
        uint64_t first = UINT64_MAX;
        for (int32_t b = 0; b < n_bin; ++b) {
            if (!need(8)) return fail("truncated BAI");
            const uint32_t bin = rd32(d.data() + p);
            const int32_t n_chunk = rdi32(d.data() + p + 4);
            p += 8;
            if (!need((size_t)n_chunk * 16)) return fail("truncated BAI");
            if (bin != 37450)
                for (int32_t c = 0; c < n_chunk; ++c) first = std::min(first, rd64(d.data() + p + (size_t)c * 16));
            else if (n_chunk == 2)  // metadata: (extent), (n_mapped, n_unmapped)
                bam->ref_records[(size_t)r] = (int64_t)(rd64(d.data() + p + 16) + rd64(d.data() + p + 24));
            p += (size_t)n_chunk * 16;
        }
        if (!need(4)) return fail("truncated BAI");
        const int32_t n_intv = rdi32(d.data() + p);
        p += 4 + (size_t)n_intv * 8;
        if (p > d.size()) return fail("truncated BAI");
        bam->ref_first_voff[(size_t)r] = first;
    }
    bam->has_index = true;
    return 0;
}

inline uint32_t cigar_ref_span(const uint8_t* cig, uint32_t n) {
    uint64_t s = 0;
    for (uint32_t i = 0; i < n; ++i) {
        const uint32_t c = rd32(cig + 4 * (size_t)i);
        const uint32_t op = c & 15u;
        if (op == 0 || op == 2 || op == 3 || op == 7 || op == 8) s += c >> 4;
    }
    return (uint32_t)std::min<uint64_t>(s, 0xFFFFFFFFu);
}

// Size of one aux field's value (after tag[2] + type[1]); 0 on malformed input.
size_t aux_value_size(const uint8_t* v, const uint8_t* end, uint8_t type) {
    switch (type) {
        case 'A': case 'c': case 'C': return 1;
        case 's': case 'S': return 2;
        case 'i': case 'I': case 'f': return 4;
        case 'Z': case 'H': {
            const uint8_t* z = (const uint8_t*)std::memchr(v, 0, (size_t)(end - v));
            return z ? (size_t)(z - v) + 1 : 0;
        }
        case 'B': {
            if (end - v < 5) return 0;
            const uint8_t sub = v[0];
            const uint32_t cnt = rd32(v + 1);
            size_t es = (sub == 'c' || sub == 'C') ? 1 : (sub == 's' || sub == 'S') ? 2 : 4;
            return 5 + (size_t)cnt * es;
        }
        default: return 0;
    }
}

struct Aux {
    const uint8_t* p;
    const uint8_t* end;
    // returns pointer to the type byte of `tag`, or nullptr
    const uint8_t* find(const char* tag) const {
        const uint8_t* q = p;
        while (q + 3 <= end) {
            const uint8_t type = q[2];
            const size_t vs = aux_value_size(q + 3, end, type);
            if (!vs || vs > (size_t)(end - q - 3)) return nullptr;
            if (q[0] == (uint8_t)tag[0] && q[1] == (uint8_t)tag[1]) return q + 2;
            q += 3 + vs;
        }
        return nullptr;
    }
};

// Iterate the records of `tid` in file order (fetch(contig) order); f(record
// bytes after block_size, block_size) for each. Returns 0 or -1 (g_err set).
template <typename F>
int for_each_record(mgp_bam* bam, int tid, F&& f) {
    uint64_t voff = bam->first_record_voff;
    if (bam->has_index) {
        voff = bam->ref_first_voff[(size_t)tid];
        if (voff == UINT64_MAX) return 0;  // no reads on this reference
    }
    Stream st;
    g_err.clear();
    if (!stream_at(bam, voff, st)) return -1;
    bool seen = false;
    for (;;) {
        if (!st.fill(4)) {
            if (!g_err.empty()) return -1;
            if (st.avail() == 0) return 0;  // clean end of file
            return fail("truncated BAM record");
        }
        const uint32_t bs = rd32(st.peek());
        if (bs < 32) return fail("corrupt BAM record (block_size < 32)");
        if (!st.fill(4 + (size_t)bs)) return fail(g_err.empty() ? "truncated BAM record body" : g_err);
        const uint8_t* r = st.peek() + 4;
        const int32_t ref = rdi32(r);
        if (ref == tid) {
            seen = true;
            const int c = f(r, bs);  // 1: continue, 0: stop, < 0: error (message set)
            if (c < 0) return -1;
            if (c == 0) return 0;
        } else if (seen || ref > tid || ref < 0) {
            return 0;  // coordinate-sorted: tid's records are contiguous
        }
        st.pos += 4 + bs;
    }
}

// Batched variant: f(recs, sizes) over every complete record of `tid` present in
// the inflated buffer at once (pointers stay valid during the call). Same return
// convention as for_each_record.
template <typename F>
int for_each_batch(mgp_bam* bam, int tid, F&& f) {
    uint64_t voff = bam->first_record_voff;
    if (bam->has_index) {
        voff = bam->ref_first_voff[(size_t)tid];
        if (voff == UINT64_MAX) return 0;
    }
    Stream st;
    g_err.clear();
    if (!stream_at(bam, voff, st)) return -1;
    bool seen = false, done = false;
    std::vector<const uint8_t*> recs;
    std::vector<uint32_t> sizes;
    while (!done) {
        if (!st.fill(4)) {
            if (!g_err.empty()) return -1;
            if (st.avail() == 0) break;
            return fail("truncated BAM record");
        }
        const uint32_t bs0 = rd32(st.peek());
        if (bs0 < 32) return fail("corrupt BAM record (block_size < 32)");
        if (!st.fill(4 + (size_t)bs0)) return fail(g_err.empty() ? "truncated BAM record body" : g_err);
        recs.clear();
        sizes.clear();
        const uint8_t* base = st.base;
        size_t p = st.pos;
        const size_t end = st.size;
        while (end - p >= 4) {
            const uint32_t bs = rd32(base + p);
            if (bs < 32) return fail("corrupt BAM record (block_size < 32)");
            if (end - p < 4 + (size_t)bs) break;
            const int32_t ref = rdi32(base + p + 4);
            if (ref == tid) {
                seen = true;
                recs.push_back(base + p + 4);
                sizes.push_back(bs);
            } else if (seen || ref > tid || ref < 0) {
                done = true;
                break;
            }
            p += 4 + (size_t)bs;
        }
        if (!recs.empty()) {
            const int c = f(recs, sizes);
            if (c < 0) return -1;
            if (c == 0) return 0;
        }
        st.pos = p;
    }
    return 0;
}

// Header-level checks of mgp_pack32_record (include/mgpileup.h) on a raw BAM record.
bool bam_packable32(int32_t pos, uint32_t l_seq, uint32_t n_cig, const uint8_t* cig) {
    if (l_seq == 0 || l_seq > MGP_PACK_MAX_LEN || n_cig > 4 || pos < 0 || pos >= 65536) return false;
    uint32_t blocks = 0;
    for (uint32_t k = 0; k < n_cig; ++k) {
        const uint32_t c = rd32(cig + 4 * k);
        if ((c >> 4) >= 4096u) return false;
        const uint32_t op = c & 15u;
        blocks += op == 0 || op == 7 || op == 8;
    }
    return blocks <= 2;
}

// Header-level and quality checks of mgp_pack_record (include/mgpileup.h) on a
// raw BAM record; the quality scan tests 8 bytes at a time.
bool bam_packable(int32_t pos, uint16_t flg, uint32_t l_seq, uint32_t n_cig, const uint8_t* cig,
                         const uint8_t* qualp) {
    if (l_seq == 0 || l_seq > MGP_PACK_MAX_LEN || n_cig > 4 || pos < -(1 << 28) || pos >= (1 << 28)) return false;
    (void)flg;
    uint32_t blocks = 0;
    for (uint32_t k = 0; k < n_cig; ++k) {
        const uint32_t c = rd32(cig + 4 * k);
        if ((c >> 4) >= 4096u) return false;
        const uint32_t op = c & 15u;
        blocks += op == 0 || op == 7 || op == 8;
    }
    if (blocks > 2) return false;
    uint32_t k = 0;
    for (; k + 8 <= l_seq; k += 8) {  // a byte > 62: its bit 7, or bit 7 of byte + 65
        uint64_t x;
        std::memcpy(&x, qualp + k, 8);
        if ((x | ((x & 0x7F7F7F7F7F7F7F7Full) + 0x4141414141414141ull)) & 0x8080808080808080ull) return false;
    }
    for (; k < l_seq; ++k)
        if (qualp[k] > 62) return false;
    return true;
}

// The batch's arrays a decode writes (the library's growable arrays for
// mgp_bam_read_ref, the caller's fixed arrays for mgp_bam_stream_next).
struct Cols {
    int32_t* start;
    int32_t* bc;
    int32_t* tlen;
    uint16_t* flag;
    uint8_t* mapq;
    uint32_t* span;
    uint64_t* roff;
    uint8_t* pay;
};

// Record decode + packing + producer placement, one chunk of records at a time:
// classify() is pass 1 (sequential, header fields only: CIGAR location with the CG
// tag, record layout, record bytes), decode() places the chunk's records (pass 1b)
// and decodes the columns and payload records on the thread pool (pass 2). A batch
// (begin_batch) may take several chunks (inflated buffers); its payload starts at 0.
// One chunk's records between the stages of the pipelined stream decode (the
// decoder's per-chunk arrays, moved out while the next chunk is walked).
struct ChunkRecs {
    std::vector<const uint8_t*> recs;
    std::vector<uint32_t> sizes;
    std::vector<uint64_t> rsz;
    std::vector<uint32_t> ncg;
    std::vector<const uint8_t*> cgp;
    std::vector<uint8_t> pkd;
    std::vector<uint64_t> dupbits;  // dup_stage's verdicts: thread t's bits at [t * words, (t + 1) * words)
    size_t k0 = 0;
    bool over = false;  // placement ran past the payload capacity (never: the batch cut bounds it)
};


struct Decoder {
    mgp_bam* b;
    mgp_host::Pool pool;
    uint64_t amask;
    bool paired;
    int32_t n_keys = 0;
    // paired placement (mgp_place_records' rule, applied chunk by chunk as records
    // stream in): open[key] = the line of cell `key` whose second half is free; key
    // n_keys collects the reads the engine's filters drop
    std::vector<uint64_t> open, open32;
    std::vector<uint8_t> fill32;
    mgp_host::DupTracker dups;  // a cell's repeated keys go with the dropped reads
    uint64_t cursor = 0;        // payload bytes placed in the batch so far
    int64_t n_tag = 0, first_tag = -1;
    // the chunk
    std::vector<const uint8_t*> recs;
    std::vector<uint32_t> sizes;
    std::vector<uint64_t> rsz;  // payload bytes of each record (then, unpaired, its offset)
    std::vector<uint32_t> ncg;  // CIGAR operations (CG tag resolved)
    std::vector<const uint8_t*> cgp;
    std::vector<uint8_t> pkd;   // record layout: 0 full, 1 packed 64-byte, 2 32-byte
    double t_p1 = 0, t_p2 = 0, t_place = 0, t_fields = 0;

    // the pool's threads (MGP_BAM_DEC_THREADS overrides the bam's count; A/B of leaving
    // cores to the placement and walk threads of the pipelined stream decode)
    // reserve: threads of the bam's count left to others (the pipelined stream decode's
    // placement and boundary-walk threads: on the box's 16-core share, 16 pool threads
    // beside them decoded C3 in 1.78 s, 14 in 1.68, 12 in 1.64)
    static int decoder_threads(mgp_bam* b, int reserve) {
        if (const char* e = std::getenv("MGP_BAM_DEC_THREADS")) {
            const long v = std::strtol(e, nullptr, 10);
            if (v > 0) return (int)v;
        }
        return std::max(1, b->n_threads - (b->n_threads > 4 ? reserve : 0));
    }
    // the next 32-byte slot of `key`: its open line's next quarter, or a new line at the
    // cursor (always 128-aligned in the paired placement); branch-free (the line opens on
    // one read in four: a branch on it mispredicted, 18 -> 15 ns per read on one core)
    uint64_t place32(size_t key) {
        const uint64_t o0 = open32[key];
        const uint32_t f0 = fill32[key];
        const bool opn = o0 == ~0ull;
        const uint64_t o = opn ? cursor : o0;
        const uint32_t f = opn ? 0u : f0;
        cursor += opn ? 128u : 0u;
        open32[key] = f == 3 ? ~0ull : o;
        fill32[key] = (uint8_t)((f + 1) & 3u);
        return o + (uint64_t)MGP_PACK32_BYTES * f;
    }
    static int32_t keys_of(mgp_bam* b) {
        int32_t n = 0;
        for (int32_t v : b->wl.vals) n = std::max(n, v + 1);
        if (b->bulk_cell >= 0) n = std::max(n, b->bulk_cell + 1);
        return n;
    }
    Decoder(mgp_bam* bam, int rec_align, int reserve = 0)
        : b(bam), pool(decoder_threads(bam, reserve)), amask((uint64_t)rec_align - 1),
          paired(bam->placement == MGP_PLACE_PAIRED),
          n_keys(paired ? keys_of(bam) : 0), dups(paired ? (size_t)keys_of(bam) : 0) {
        open.assign(paired ? (size_t)n_keys + 1 : 0, ~0ull);
        open32.assign(paired ? (size_t)n_keys + 1 : 0, ~0ull);
        fill32.assign(paired ? (size_t)n_keys + 1 : 0, 0);
    }
    void begin_batch() {
        cursor = 0;
        std::fill(open.begin(), open.end(), ~0ull);
        std::fill(open32.begin(), open32.end(), ~0ull);
        std::fill(fill32.begin(), fill32.end(), (uint8_t)0);
    }
    void clear_chunk() {
        recs.clear();
        sizes.clear();
        rsz.clear();
        ncg.clear();
        cgp.clear();
        pkd.clear();
    }
    // payload bytes a classified record takes at most in its batch, lines included
    // (a batch may also leave one partly filled line per key and layout: callers add
    // 2 x 128 x (n_keys + 1))
    uint64_t worst(size_t i) const {
        if (!paired) return (rsz[i] + amask) & ~amask;
        return pkd[i] ? rsz[i] : ((rsz[i] + 127) & ~127ull) + 127;
    }
    uint64_t line_slack() const { return paired ? 2ull * 128ull * ((uint64_t)n_keys + 1) : 0ull; }

    // pass 1 over the chunk's records (recs/sizes filled by the caller), on the pool;
    // false on a malformed record
    bool classify_all() {
        const size_t m = recs.size();
        rsz.resize(m);
        ncg.resize(m);
        cgp.resize(m);
        pkd.resize(m);
        const int tn = (int)std::max<size_t>(1, std::min<size_t>((size_t)pool.size(), m / 8192 + 1));
        std::atomic<bool> ok{true};
        std::string msg;
        std::mutex mu;
        pool.run(tn, [&](int t) {
            const size_t lo = m * (size_t)t / (size_t)tn, hi = m * (size_t)(t + 1) / (size_t)tn;
            for (size_t i = lo; i < hi; ++i)
                if (!classify_at(i)) {
                    std::lock_guard<std::mutex> g(mu);
                    if (ok) msg = g_err;
                    ok = false;
                    return;
                }
        });
        if (!ok) g_err = msg;
        return ok;
    }
    void truncate(size_t m) {
        recs.resize(m);
        sizes.resize(m);
        rsz.resize(m);
        ncg.resize(m);
        cgp.resize(m);
        pkd.resize(m);
    }
    // pass 1 for record i of the chunk; false on a malformed record
    bool classify_at(size_t i) {
        const uint8_t* r = recs[i];
        const uint32_t size = sizes[i];
        const uint8_t l_name = r[8];
        uint32_t n_cig = rd16(r + 12);
        const uint32_t l_seq = rd32(r + 16);
        const uint8_t* cigp = r + 32 + l_name;
        const uint8_t* auxp = cigp + 4 * (size_t)n_cig + ((size_t)l_seq + 1) / 2 + l_seq;
        if (auxp > r + size) return fail("corrupt BAM record (fields exceed block_size)"), false;
        const uint8_t* cig = cigp;
        // CIGAR with > 65535 operations lives in the CG:B,I tag (placeholder kSmN)
        if (n_cig == 2 && (rd32(cigp) & 15u) == 4 && (rd32(cigp) >> 4) == l_seq && (rd32(cigp + 4) & 15u) == 3) {
            Aux aux{auxp, r + size};
            const uint8_t* t = aux.find("CG");
            if (t && t[0] == 'B' && (t[1] == 'I' || t[1] == 'i')) {
                n_cig = rd32(t + 2);
                cig = t + 6;
            }
        }
        if (n_cig > 0xFFFF)
            return fail("CIGAR with more than 65535 operations is not supported by the record format"), false;
        const uint8_t* qualp = cigp + 4 * (size_t)rd16(r + 12) + ((size_t)l_seq + 1) / 2;
        const bool seqqual = l_seq != 0 && qualp[0] != 0xFF;  // else NOSEQQUAL: never packed
        const uint8_t pk = (b->pack32 && seqqual && bam_packable32(rdi32(r + 4), l_seq, n_cig, cig)) ? 2
                           : (b->pack && bam_packable(rdi32(r + 4), rd16(r + 14), l_seq, n_cig, cig, qualp)) ? 1 : 0;
        ncg[i] = n_cig;
        cgp[i] = cig;
        pkd[i] = pk;
        rsz[i] = pk == 2 ? (uint64_t)MGP_PACK32_BYTES
                 : pk ? (uint64_t)MGP_PACK_BYTES
                      : (uint64_t)mgp_cigar_offset(l_seq) + 4ull * n_cig;
        return true;
    }

    // one record: decode (do_fields: the SoA columns, barcode lookup included) and
    // pack (do_rec: the payload record at offset off) at index k
    void decode_one(const Cols& c, const uint8_t* r, uint32_t bs, size_t k, uint64_t off, uint32_t n_cig,
                    const uint8_t* cig, int pk, int64_t& tags, int64_t& first, int64_t gidx, bool do_fields,
                    bool do_rec) const {
        const uint8_t* end = r + bs;
        const int32_t pos = rdi32(r + 4);
        const uint8_t l_name = r[8];
        const uint8_t mq = r[9];
        const uint16_t flg = rd16(r + 14);
        const uint32_t l_seq = rd32(r + 16);
        const int32_t tl = rdi32(r + 28);
        const uint8_t* seqp = r + 32 + l_name + 4 * (size_t)rd16(r + 12);
        const uint8_t* qualp = seqp + ((size_t)l_seq + 1) / 2;
        const uint8_t* auxp = qualp + l_seq;
        uint16_t fl = flg & 0x0FFF;
        if (l_seq == 0 || qualp[0] == 0xFF) fl |= MGP_FLAG_NOSEQQUAL;
        if (pk == 1) fl |= MGP_FLAG_PACKED;
        if (pk == 2) fl |= MGP_FLAG_PACK32;
        if (do_fields) {
            Aux aux{auxp, end};
            int32_t bcv = -1;
            const uint8_t* t = aux.find(b->tag);
            if (t) {
                ++tags;
                if (first < 0) first = gidx;
                if (t[0] == 'Z' || t[0] == 'H') {  // get_tag() -> str; numeric tags never match
                    const char* sv = (const char*)t + 1;
                    bcv = b->wl.get(sv, std::strlen(sv));
                } else if (t[0] == 'A') {
                    bcv = b->wl.get((const char*)t + 1, 1);
                }
            }
            if (b->bulk_cell >= 0) bcv = b->bulk_cell;
            c.start[k] = pos;
            c.bc[k] = bcv;
            c.tlen[k] = tl;
            c.flag[k] = fl;
            c.mapq[k] = mq;
            c.span[k] = std::max(cigar_ref_span(cig, n_cig), l_seq);
            c.roff[k] = off;
        }
        if (!do_rec) return;
        uint8_t* rec = c.pay + off;
        if (pk == 2) {
            uint32_t cw[4] = {0, 0, 0, 0};
            for (uint32_t q = 0; q < n_cig; ++q) cw[q] = rd32(cig + 4 * q);
            const uint64_t size = ((uint64_t)MGP_PACK32_BYTES + amask) & ~amask;
            if (size > MGP_PACK32_BYTES && !paired) std::memset(rec + MGP_PACK32_BYTES, 0, size - MGP_PACK32_BYTES);
            mgp_host::pack32_record_fast(pos, l_seq, fl, n_cig, cw, seqp, qualp, b->pack32_minq, b->pack32_dist,
                                         rec);  // all 32 B
        } else if (pk) {
            uint32_t cw[4] = {0, 0, 0, 0};
            for (uint32_t q = 0; q < n_cig; ++q) cw[q] = rd32(cig + 4 * q);
            const uint64_t size = ((uint64_t)MGP_PACK_BYTES + amask) & ~amask;
            if (size > MGP_PACK_BYTES && !paired) std::memset(rec + MGP_PACK_BYTES, 0, size - MGP_PACK_BYTES);
            mgp_host::pack64_record_fast(pos, l_seq, fl, n_cig, cw, seqp, qualp, end, rec);  // all 64 bytes
        } else {
            const uint32_t soff = mgp_seq_offset(l_seq);
            const uint32_t coff = mgp_cigar_offset(l_seq);
            const uint64_t size = ((uint64_t)coff + 4ull * n_cig + (paired ? 127u : amask)) & ~(paired ? 127ull : amask);
            std::memset(rec, 0, size);
            std::memcpy(rec, &pos, 4);
            std::memcpy(rec + 4, &l_seq, 4);
            const uint16_t nc16 = (uint16_t)n_cig;
            std::memcpy(rec + 8, &nc16, 2);
            std::memcpy(rec + 10, &fl, 2);
            std::memcpy(rec + 12, &coff, 4);
            if (l_seq) {
                std::memcpy(rec + 16, qualp, l_seq);
                std::memcpy(rec + soff, seqp, ((size_t)l_seq + 1) / 2);
            }
            if (n_cig) std::memcpy(rec + coff, cig, 4 * (size_t)n_cig);
        }
    }

    // Decode the chunk's records at index k0 of the batch (global record index gidx0),
    // payload appended at `cursor`. reserve(kn, pay_end) makes room for kn columns and
    // pay_end payload bytes (+256), then cols() are the arrays; false = out of memory.
    template <class Reserve, class GetCols>
    int decode(size_t k0, int64_t gidx0, Reserve&& reserve, GetCols&& cols) {
        const int nt = pool.size();
        const double tp1 = now_s();
        const size_t m = recs.size();
        if (!m) return 0;
        const size_t kn = k0 + m;
        // unpaired: dense offsets from the cursor (records are rec_align-sized)
        uint64_t end = cursor;
        if (!paired) {
            for (size_t i = 0; i < m; ++i) {
                const uint64_t off = (end + amask) & ~amask;
                end = off + ((rsz[i] + amask) & ~amask);
                rsz[i] = off;
            }
        }
        if (!reserve(kn, paired ? cursor : end)) return fail("out of host memory"), -1;
        const double tp2 = now_s();
        t_p1 += tp2 - tp1;
        const int tn = (int)std::max<size_t>(1, std::min<size_t>((size_t)nt, m / 4096 + 1));
        std::vector<int64_t> tags((size_t)tn, 0), firsts((size_t)tn, -1);
        auto run_pass = [&](const Cols& c, bool do_fields, bool do_rec) {
            pool.run(tn, [&](int t) {
                const size_t lo = m * (size_t)t / (size_t)tn, hi = m * (size_t)(t + 1) / (size_t)tn;
                for (size_t i = lo; i < hi; ++i)
                    decode_one(c, recs[i], sizes[i], k0 + i, paired ? c.roff[k0 + i] : rsz[i], ncg[i], cgp[i],
                               (int)pkd[i], tags[(size_t)t], firsts[(size_t)t], gidx0 + (int64_t)i, do_fields, do_rec);
                _mm_sfence();  // (the records' non-temporal stores)
            });
        };
        if (!paired) {
            run_pass(cols(), true, true);
            cursor = end;
        } else {
            double tpl = 0;
            {
                const Cols c = cols();
                const double tf = now_s();
                run_pass(c, true, false);
                t_fields += now_s() - tf;
                tpl = now_s();
                // pass 1b: which half-line each record takes (mgp_place_records' rule)
                const uint16_t drop = MGP_FLAG_UNMAPPED | MGP_FLAG_SECONDARY | MGP_FLAG_SUPPLEMENTARY;
                for (size_t i = 0; i < m; ++i) {
                    const size_t k = k0 + i;
                    if (!pkd[i]) {
                        cursor = (cursor + 127) & ~127ull;
                        c.roff[k] = cursor;
                        cursor += (rsz[i] + 127) & ~127ull;
                        continue;
                    }
                    const int32_t cc = c.bc[k];
                    size_t key = (cc >= 0 && cc < n_keys && !(c.flag[k] & drop)) ? (size_t)cc : (size_t)n_keys;
                    if (key < (size_t)n_keys &&
                        dups.repeat(key, c.start[k], (c.flag[k] & MGP_FLAG_REVERSE) != 0, c.tlen[k]))
                        key = (size_t)n_keys;
                    if (pkd[i] == 2) {  // four 32-byte records of one key per line
                        c.roff[k] = place32(key);
                        continue;
                    }
                    if (open[key] != ~0ull) {
                        c.roff[k] = open[key] + MGP_PACK_BYTES;
                        open[key] = ~0ull;
                    } else {
                        cursor = (cursor + 127) & ~127ull;
                        c.roff[k] = open[key] = cursor;
                        cursor += 128;
                    }
                }
            }
            t_place += now_s() - tpl;
            if (!reserve(kn, cursor)) return fail("out of host memory"), -1;
            const Cols c = cols();
            // second halves of lines that stay open: zero (a later chunk may still fill
            // them; the others are fully written); only lines of this chunk can be open
            // and unwritten, lines of earlier chunks were zeroed then
            for (uint64_t o : open)
                if (o != ~0ull) std::memset(c.pay + o + MGP_PACK_BYTES, 0, MGP_PACK_BYTES);
            for (size_t key = 0; key < open32.size(); ++key)
                if (open32[key] != ~0ull)
                    std::memset(c.pay + open32[key] + (uint64_t)MGP_PACK32_BYTES * fill32[key], 0,
                                (uint64_t)MGP_PACK32_BYTES * (4u - fill32[key]));
            run_pass(c, false, true);
        }
        for (int t = 0; t < tn; ++t) {
            n_tag += tags[(size_t)t];
            if (first_tag < 0 && firsts[(size_t)t] >= 0) first_tag = firsts[(size_t)t];
        }
        t_p2 += now_s() - tp2;
        return 0;
    }

    // ---- the pipelined stream decode (paired placement): fields of chunk j on the
    // pool, then chunk j's placement on a thread of its own while the pool walks,
    // classifies and decodes the fields of chunk j + 1, then chunk j's records.
    // fields_stage: the current chunk's columns at k0 (no payload yet)
    void fields_stage(size_t k0, int64_t gidx0, const Cols& c) {
        const double t0 = now_s();
        const size_t m = recs.size();
        const int tn = (int)std::max<size_t>(1, std::min<size_t>((size_t)pool.size(), m / 4096 + 1));
        std::vector<int64_t> tags((size_t)tn, 0), firsts((size_t)tn, -1);
        pool.run(tn, [&](int t) {
            const size_t lo = m * (size_t)t / (size_t)tn, hi = m * (size_t)(t + 1) / (size_t)tn;
            for (size_t i = lo; i < hi; ++i)
                decode_one(c, recs[i], sizes[i], k0 + i, 0, ncg[i], cgp[i], (int)pkd[i], tags[(size_t)t],
                           firsts[(size_t)t], gidx0 + (int64_t)i, true, false);
        });
        for (int t = 0; t < tn; ++t) {
            n_tag += tags[(size_t)t];
            if (first_tag < 0 && firsts[(size_t)t] >= 0) first_tag = firsts[(size_t)t];
        }
        t_fields += now_s() - t0;
    }
    // pass 1 and the columns of the current chunk at k0 in one pool pass; hastag[i]: the
    // record carries the barcode tag (counted by count_tags for the records the batch keeps)
    std::vector<uint8_t> hastag;
    bool classify_fields_all(size_t k0, int64_t gidx0, const Cols& c) {
        const double t0 = now_s();
        const size_t m = recs.size();
        rsz.resize(m);
        ncg.resize(m);
        cgp.resize(m);
        pkd.resize(m);
        hastag.resize(m);
        const int tn = (int)std::max<size_t>(1, std::min<size_t>((size_t)pool.size(), m / 4096 + 1));
        std::atomic<bool> ok{true};
        std::string msg;
        std::mutex mu;
        pool.run(tn, [&](int t) {
            const size_t lo = m * (size_t)t / (size_t)tn, hi = m * (size_t)(t + 1) / (size_t)tn;
            for (size_t i = lo; i < hi; ++i) {
                if (!classify_at(i)) {
                    std::lock_guard<std::mutex> g(mu);
                    if (ok) msg = g_err;
                    ok = false;
                    return;
                }
                int64_t tg = 0, fs = -1;
                decode_one(c, recs[i], sizes[i], k0 + i, 0, ncg[i], cgp[i], (int)pkd[i], tg, fs, gidx0 + (int64_t)i,
                           true, false);
                hastag[i] = tg != 0;
            }
        });
        if (!ok) g_err = msg;
        t_fields += now_s() - t0;
        return ok;
    }
    // BAM-order decode in one pool pass: pass 1, the columns and each record written at
    // the cursor + 64 x its index in the chunk, the offset it takes when every record of
    // the chunk is a 64-byte slot (packed, rec_align 64: the speculation); all64 says
    // whether it held (else the caller places and writes the chunk's records again).
    // Records past the payload capacity are not written (the batch cut drops them).
    bool classify_fields_records_all(size_t k0, int64_t gidx0, const Cols& c, uint64_t cap_payload, bool& all64) {
        const double t0 = now_s();
        const size_t m = recs.size();
        rsz.resize(m);
        ncg.resize(m);
        cgp.resize(m);
        pkd.resize(m);
        hastag.resize(m);
        const int tn = (int)std::max<size_t>(1, std::min<size_t>((size_t)pool.size(), m / 4096 + 1));
        std::atomic<bool> ok{true}, spec{amask == 63};
        std::string msg;
        std::mutex mu;
        const uint64_t base = cursor;
        pool.run(tn, [&](int t) {
            const size_t lo = m * (size_t)t / (size_t)tn, hi = m * (size_t)(t + 1) / (size_t)tn;
            bool sp = spec.load(std::memory_order_relaxed);
            for (size_t i = lo; i < hi; ++i) {
                if (!classify_at(i)) {
                    std::lock_guard<std::mutex> g(mu);
                    if (ok) msg = g_err;
                    ok = false;
                    return;
                }
                int64_t tg = 0, fs = -1;
                sp = sp && pkd[i] == 1;
                const uint64_t off = base + 64ull * i;
                const bool rec = sp && off + 64 + 256 <= cap_payload;
                decode_one(c, recs[i], sizes[i], k0 + i, off, ncg[i], cgp[i], (int)pkd[i], tg, fs, gidx0 + (int64_t)i,
                           true, rec);
                hastag[i] = tg != 0;
            }
            _mm_sfence();
            if (!sp) spec.store(false, std::memory_order_relaxed);
        });
        if (!ok) g_err = msg;
        all64 = spec.load();
        t_fields += now_s() - t0;
        return ok;
    }
    void count_tags(int64_t gidx0) {
        const size_t m = recs.size();
        for (size_t i = 0; i < m; ++i)
            if (hastag[i]) {
                ++n_tag;
                if (first_tag < 0) first_tag = gidx0 + (int64_t)i;
            }
    }
    // the current chunk's arrays into q (the decoder's are then empty, capacity kept)
    void move_chunk(ChunkRecs& q, size_t k0) {
        q.recs.swap(recs);
        q.sizes.swap(sizes);
        q.rsz.swap(rsz);
        q.ncg.swap(ncg);
        q.cgp.swap(cgp);
        q.pkd.swap(pkd);
        q.dupbits.swap(dupbits);
        q.k0 = k0;
        q.over = false;
        clear_chunk();
    }
    // The duplicate-key check of the current chunk (DupTracker::repeat in BAM order per
    // cell) on the pool, cells dealt to the threads by id: a cell's reads stay in order
    // on one thread, and each thread writes its verdicts to bits of its own. The serial
    // placement then only reads them (it was the stream decode's critical path at C4).
    // (The reads are first dealt to their owners, T ranges counted then listed in
    // parallel, so each thread walks only its own reads, still in BAM order.)
    std::vector<uint64_t> dupbits;
    std::vector<uint32_t> dup_idx;
    std::vector<size_t> dup_at;
    void dup_stage(size_t k0, const Cols& c) {
        const double t0 = now_s();
        const size_t m = recs.size(), words = (m + 63) / 64;
        const int T = pool.size();
        dupbits.assign((size_t)T * words, 0ull);
        const uint16_t drop = MGP_FLAG_UNMAPPED | MGP_FLAG_SECONDARY | MGP_FLAG_SUPPLEMENTARY;
        auto owner = [&](size_t i) -> int {  // the thread checking read i, -1: no check
            const size_t k = k0 + i;
            const int32_t cc = c.bc[k];
            if (cc < 0 || cc >= n_keys || !pkd[i] || (c.flag[k] & drop)) return -1;
            return cc % T;
        };
        // counts per (range r, owner t), then every (r, t) block's place in the owner-major list
        dup_at.assign((size_t)T * T + 1, 0);
        pool.run(T, [&](int r) {
            const size_t lo = m * (size_t)r / (size_t)T, hi = m * (size_t)(r + 1) / (size_t)T;
            size_t* cnt = dup_at.data() + (size_t)r * T;
            for (size_t i = lo; i < hi; ++i) {
                const int o = owner(i);
                if (o >= 0) ++cnt[o];
            }
        });
        std::vector<size_t> start((size_t)T * T + 1);
        size_t tot = 0;
        for (int t = 0; t < T; ++t)
            for (int r = 0; r < T; ++r) {
                start[(size_t)r * T + t] = tot;
                tot += dup_at[(size_t)r * T + t];
            }
        std::vector<size_t> seg((size_t)T + 1);  // owner t's reads: [seg[t], seg[t + 1])
        for (int t = 0; t < T; ++t) seg[(size_t)t] = start[(size_t)t];
        seg[(size_t)T] = tot;
        dup_idx.resize(std::max<size_t>(tot, 1));
        pool.run(T, [&](int r) {
            const size_t lo = m * (size_t)r / (size_t)T, hi = m * (size_t)(r + 1) / (size_t)T;
            size_t* at = start.data() + (size_t)r * T;
            for (size_t i = lo; i < hi; ++i) {
                const int o = owner(i);
                if (o >= 0) dup_idx[at[o]++] = (uint32_t)i;
            }
        });
        pool.run(T, [&](int t) {
            uint64_t* bits = dupbits.data() + (size_t)t * words;
            for (size_t x = seg[(size_t)t]; x < seg[(size_t)t + 1]; ++x) {
                const size_t i = dup_idx[x], k = k0 + i;
                if (dups.repeat((size_t)c.bc[k], c.start[k], (c.flag[k] & MGP_FLAG_REVERSE) != 0, c.tlen[k]))
                    bits[i >> 6] |= 1ull << (i & 63);
            }
        });
        t_dups += now_s() - t0;
    }
    double t_dups = 0;
    // placement of chunk q (serial: the line state carries over in BAM order), then the
    // free slots of the lines left open are zeroed (a later chunk may fill them; every
    // other slot gets its record)
    void place_stage(ChunkRecs& q, const Cols& c, uint64_t cap_payload) {
        const double t0 = now_s();
        const uint16_t drop = MGP_FLAG_UNMAPPED | MGP_FLAG_SECONDARY | MGP_FLAG_SUPPLEMENTARY;
        const size_t m = q.recs.size(), words = (m + 63) / 64;
        const int T = pool.size();
        for (size_t i = 0; i < m; ++i) {
            const size_t k = q.k0 + i;
            if ((k & 15) == 0) {  // the columns other cores just wrote: lines well ahead in flight
                __builtin_prefetch(c.bc + k + 512);
                __builtin_prefetch(c.start + k + 512);
                __builtin_prefetch(c.tlen + k + 512);
                __builtin_prefetch(c.flag + k + 512);
                __builtin_prefetch(c.roff + k + 512, 1);
                __builtin_prefetch(c.roff + k + 520, 1);
            }
            if (!q.pkd[i]) {
                cursor = (cursor + 127) & ~127ull;
                c.roff[k] = cursor;
                cursor += (q.rsz[i] + 127) & ~127ull;
                continue;
            }
            const int32_t cc = c.bc[k];
            size_t key = (cc >= 0 && cc < n_keys && !(c.flag[k] & drop)) ? (size_t)cc : (size_t)n_keys;
            // (dup_stage's verdict: the bits of the thread that owned the cell)
            if (key < (size_t)n_keys && (q.dupbits[(size_t)(cc % T) * words + (i >> 6)] >> (i & 63)) & 1ull)
                key = (size_t)n_keys;
            if (q.pkd[i] == 2) {
                c.roff[k] = place32(key);
                continue;
            }
            if (open[key] != ~0ull) {
                c.roff[k] = open[key] + MGP_PACK_BYTES;
                open[key] = ~0ull;
            } else {
                cursor = (cursor + 127) & ~127ull;
                c.roff[k] = open[key] = cursor;
                cursor += 128;
            }
        }
        if (cursor + 256 > cap_payload) {
            q.over = true;
        } else {
            for (uint64_t o : open)
                if (o != ~0ull) std::memset(c.pay + o + MGP_PACK_BYTES, 0, MGP_PACK_BYTES);
            for (size_t key = 0; key < open32.size(); ++key)
                if (open32[key] != ~0ull)
                    std::memset(c.pay + open32[key] + (uint64_t)MGP_PACK32_BYTES * fill32[key], 0,
                                (uint64_t)MGP_PACK32_BYTES * (4u - fill32[key]));
        }
        t_place += now_s() - t0;
    }
    // chunk q's payload records at their placed offsets, on the pool
    void records_stage(const ChunkRecs& q, const Cols& c) {
        const double t0 = now_s();
        const size_t m = q.recs.size();
        const int tn = (int)std::max<size_t>(1, std::min<size_t>((size_t)pool.size(), m / 4096 + 1));
        pool.run(tn, [&](int t) {
            const size_t lo = m * (size_t)t / (size_t)tn, hi = m * (size_t)(t + 1) / (size_t)tn;
            int64_t tg = 0, fs = -1;  // (tags are counted by fields_stage)
            for (size_t i = lo; i < hi; ++i)
                decode_one(c, q.recs[i], q.sizes[i], q.k0 + i, c.roff[q.k0 + i], q.ncg[i], q.cgp[i], (int)q.pkd[i],
                           tg, fs, 0, false, true);
            _mm_sfence();
        });
        t_recs += now_s() - t0;
    }
    double t_recs = 0;
    // BAM-order placement of the current chunk at k0: each record at the cursor in
    // rec_align-sized slots (a running sum: the sizes come from pass 1)
    void dense_offsets(size_t k0, const Cols& c) {
        const size_t m = recs.size();
        for (size_t i = 0; i < m; ++i) {
            const uint64_t off = (cursor + amask) & ~amask;
            c.roff[k0 + i] = off;
            cursor = off + ((rsz[i] + amask) & ~amask);
        }
    }
    // the current chunk's payload records at their offsets, on the pool
    void records_inline(size_t k0, const Cols& c) {
        const double t0 = now_s();
        const size_t m = recs.size();
        const int tn = (int)std::max<size_t>(1, std::min<size_t>((size_t)pool.size(), m / 4096 + 1));
        pool.run(tn, [&](int t) {
            const size_t lo = m * (size_t)t / (size_t)tn, hi = m * (size_t)(t + 1) / (size_t)tn;
            int64_t tg = 0, fs = -1;  // (tags are counted by count_tags)
            for (size_t i = lo; i < hi; ++i)
                decode_one(c, recs[i], sizes[i], k0 + i, c.roff[k0 + i], ncg[i], cgp[i], (int)pkd[i], tg, fs, 0, false,
                           true);
            _mm_sfence();
        });
        t_recs += now_s() - t0;
    }
};

// Growable malloc'd array (handed to the caller as is: no final copy).
template <typename T>
struct Grow {
    T* p = nullptr;
    size_t n = 0, cap = 0;
    bool reserve(size_t want) {
        if (want <= cap) return true;
        size_t nc = std::max(want, cap + cap / 2 + 1024);
        T* q = (T*)std::realloc(p, nc * sizeof(T));
        if (!q) return false;
        p = q;
        cap = nc;
        return true;
    }
};

}  // namespace

extern "C" {

const char* mgp_host_last_error(void) { return g_err.c_str(); }
void mgp_host_buf_free(void* p) { std::free(p); }

int mgp_bam_open(const char* path, int n_threads, mgp_bam** out) {
    g_err.clear();
    if (!path || !out) return fail("null argument");
    mgp_bam* b = new mgp_bam();
    b->path = path;
    b->fd = ::open(path, O_RDONLY);
    if (b->fd < 0) {
        delete b;
        return fail(std::string("cannot open ") + path + ": " + std::strerror(errno));
    }
    b->file_size = (int64_t)::lseek(b->fd, 0, SEEK_END);
    unsigned hc = std::thread::hardware_concurrency();
    b->n_threads = n_threads > 0 ? n_threads : (int)std::max(1u, std::min(hc, 16u));
    if (parse_header(b) != 0 || load_index(b) != 0) {
        ::close(b->fd);
        delete b;
        return -1;
    }
    *out = b;
    return 0;
}

void mgp_bam_close(mgp_bam* b) {
    if (!b) return;
    if (b->fd >= 0) ::close(b->fd);
    delete b;
}

int mgp_bam_n_refs(mgp_bam* b) { return b ? (int)b->ref_names.size() : 0; }
const char* mgp_bam_ref_name(mgp_bam* b, int tid) {
    return (b && tid >= 0 && tid < (int)b->ref_names.size()) ? b->ref_names[(size_t)tid].c_str() : nullptr;
}
int64_t mgp_bam_ref_len(mgp_bam* b, int tid) {
    return (b && tid >= 0 && tid < (int)b->ref_lens.size()) ? b->ref_lens[(size_t)tid] : -1;
}
int mgp_bam_has_index(mgp_bam* b) { return b && b->has_index ? 1 : 0; }

int mgp_bam_set_barcodes(mgp_bam* b, const char* tag, const char* const* barcodes, int n) {
    if (!b || !tag || std::strlen(tag) != 2 || n < 0 || (n && !barcodes)) return fail("bad barcode arguments");
    b->tag[0] = tag[0];
    b->tag[1] = tag[1];
    std::vector<std::string> k((size_t)n);
    std::vector<int32_t> v((size_t)n);
    for (int i = 0; i < n; ++i) {
        k[(size_t)i] = barcodes[i];
        v[(size_t)i] = i;
    }
    b->wl.build(k, v);
    b->bulk_cell = -1;
    return 0;
}

int mgp_bam_set_bulk(mgp_bam* b, int32_t cell) {
    if (!b || cell < -1) return fail("bad bulk arguments");
    b->bulk_cell = cell;
    return 0;
}

int mgp_bam_set_placement(mgp_bam* b, int mode) {
    if (!b) return fail("null argument");
    if (mode != MGP_PLACE_DENSE && mode != MGP_PLACE_PAIRED) return fail("unknown placement");
    b->placement = mode;
    return 0;
}

int mgp_bam_set_pack(mgp_bam* b, int pack) {
    if (!b) return fail("null argument");
    b->pack = pack != 0;
    if (!b->pack) b->pack32 = false;
    return 0;
}

int mgp_bam_set_pack32(mgp_bam* b, int on, int min_baseq, int min_dist) {
    if (!b) return fail("null argument");
    if (on && (min_baseq < -128 || min_baseq > 127 || min_dist > 15))
        return fail("32-byte records need min_baseq in [-128, 127] and min_dist_from_end <= 15");
    b->pack32 = on != 0;
    b->pack32_minq = min_baseq;
    b->pack32_dist = min_dist;
    if (b->pack32) b->pack = true;
    return 0;
}

int mgp_bam_read_ref(mgp_bam* b, int tid, int rec_align, mgp_bam_batch* out) {
    g_err.clear();
    if (!b || !out) return fail("null argument");
    if (tid < 0 || tid >= (int)b->ref_names.size()) return fail("reference id out of range");
    if (rec_align < 16 || rec_align > 4096 || (rec_align & (rec_align - 1))) return fail("bad rec_align");
    std::memset(out, 0, sizeof(*out));
    out->first_tag_index = -1;
    Grow<int32_t> G_start, G_bc, G_tlen;
    Grow<uint16_t> G_flag;
    Grow<uint8_t> G_mapq, G_pay;
    Grow<uint32_t> G_span;
    Grow<uint64_t> G_roff;
    const int nt = std::max(1, b->n_threads);
    const double t_begin = now_s();
    t_inflate = t_pread = 0;
    Decoder dec(b, rec_align);
    dec.begin_batch();
    auto reserve = [&](size_t kn, uint64_t pay_end) {
        return G_start.reserve(kn) && G_bc.reserve(kn) && G_tlen.reserve(kn) && G_flag.reserve(kn) &&
               G_mapq.reserve(kn) && G_span.reserve(kn) && G_roff.reserve(kn) && G_pay.reserve(pay_end + 256);
    };
    auto cols = [&]() { return Cols{G_start.p, G_bc.p, G_tlen.p, G_flag.p, G_mapq.p, G_span.p, G_roff.p, G_pay.p}; };
    const int rc = for_each_batch(b, tid, [&](const std::vector<const uint8_t*>& recs,
                                              const std::vector<uint32_t>& sizes) -> int {
        const double tp1 = now_s();
        dec.clear_chunk();
        dec.recs = recs;
        dec.sizes = sizes;
        if (!dec.classify_all()) return -1;
        dec.t_p1 += now_s() - tp1;
        const size_t k0 = G_start.n;
        if (dec.decode(k0, (int64_t)k0, reserve, cols) != 0) return -1;
        G_start.n = G_bc.n = G_tlen.n = G_flag.n = G_mapq.n = G_span.n = G_roff.n = k0 + recs.size();
        G_pay.n = dec.cursor;
        return 1;
    });
    if (std::getenv("MGP_HOST_PROFILE"))
        std::fprintf(stderr, "[mgp_bam_read_ref] %zu records, %d threads: total %.3f s = pread %.3f + inflate %.3f + "
                     "scan/sizes %.3f + decode %.3f (fields %.3f, placement %.3f) (+ rest)\n", G_start.n, nt,
                     now_s() - t_begin, t_pread, t_inflate, dec.t_p1, dec.t_p2, dec.t_fields, dec.t_place);
    auto release = [&]() {
        std::free(G_start.p); std::free(G_bc.p); std::free(G_tlen.p); std::free(G_flag.p);
        std::free(G_mapq.p); std::free(G_span.p); std::free(G_roff.p); std::free(G_pay.p);
    };
    if (rc != 0) {
        release();
        return -1;
    }
    // at least one element everywhere; >= 256 bytes of payload slack for vector over-reads
    if (!reserve(std::max<size_t>(G_start.n, 1), G_pay.n)) {
        release();
        return fail("out of host memory");
    }
    std::memset(G_pay.p + G_pay.n, 0, 256);
    out->n_reads = (int64_t)G_start.n;
    out->start = G_start.p;
    out->bc = G_bc.p;
    out->tlen = G_tlen.p;
    out->flag = G_flag.p;
    out->mapq = G_mapq.p;
    out->span = G_span.p;
    out->rec_off = G_roff.p;
    out->payload = G_pay.p;
    out->payload_bytes = (int64_t)G_pay.n;
    out->n_with_tag = dec.n_tag;
    out->first_tag_index = dec.first_tag;
    return 0;
}

// ---- streaming decode (one pass in batches, readers.py:84-93) -------------------
struct mgp_bam_stream {
    mgp_bam* bam = nullptr;
    int tid = 0;
    Stream st;
    bool seen = false, done = false;
    Decoder dec;
    int64_t decoded = 0;  // records handed out so far
    std::vector<size_t> offs;  // the chunk's record offsets in the stream buffer
    double t_fill = 0, t_walk = 0, t_class = 0, t_open = 0, t_wait = 0;  // MGP_HOST_PROFILE
    double t_list = 0;
    int64_t n_listed = 0, n_walked = 0;  // chunks whose boundaries came from the prefetch walk / were walked here
    // the pipelined decode (paired placement; MGP_BAM_PIPELINE=0 turns it off): the
    // chunk whose placement runs on `placer` and whose records are still to be written
    static bool pipe_env() {
        const char* e = std::getenv("MGP_BAM_PIPELINE");
        return !e || std::strtol(e, nullptr, 10) != 0;
    }
    bool pipe = true, fuse = true;
    // BAM-order records (no cell pairing: the engine pairs a dense batch of 64-byte
    // records on the device, mgp_push_batch): pass 1 and the columns in one pool pass,
    // the offsets by a running sum, the records in a second pool pass; no placement
    // thread, no duplicate-key stage (MGP_BAM_DENSE_FUSE=0: the two-pass decode)
    bool dense_fuse = false;
    ChunkRecs pend;
    bool pending = false;
    Worker placer;
    mgp_bam_stream(mgp_bam* b, int rec_align)
        : bam(b), dec(b, rec_align, b->placement == MGP_PLACE_PAIRED && pipe_env() ? 2 : 0) {
        t_open = now_s();
        pipe = pipe_env() && dec.paired;
        st.hold = pipe;
        const char* ef = std::getenv("MGP_BAM_FUSE");  // pass 1 and the columns in one pass (pipelined)
        fuse = pipe && (!ef || std::strtol(ef, nullptr, 10) != 0);
        const char* ed = std::getenv("MGP_BAM_DENSE_FUSE");
        dense_fuse = !dec.paired && (!ed || std::strtol(ed, nullptr, 10) != 0);
    }
    ~mgp_bam_stream() {
        if (pending) placer.wait();  // (an abandoned batch: its placement may still run)
        if (std::getenv("MGP_HOST_PROFILE") && st.pf) st.pf->join();  // (its counters, once its thread has ended)
        if (std::getenv("MGP_HOST_PROFILE"))
            std::fprintf(stderr,
                         "[mgp_bam_stream] %lld records, %d threads%s: open %.3f s; waiting for inflated chunks %.3f, "
                         "record walk %.3f (listed %.3f; prefetch: read %.3f, inflate %.3f, walk %.3f; %lld + %lld chunks), "
                         "classify %.3f, fields %.3f, "
                         "duplicate keys %.3f, placement %.3f (waited for %.3f), records %.3f\n",
                         (long long)decoded, dec.pool.size(), pipe ? ", pipelined" : dense_fuse ? ", BAM order fused" : "",
                         now_s() - t_open, t_fill,
                         t_walk, t_list, st.pf ? st.pf->t_pread : 0.0, st.pf ? st.pf->t_inflate : 0.0,
                         st.pf ? st.pf->t_walk : 0.0, (long long)n_listed, (long long)n_walked, t_class, dec.t_fields,
                         dec.t_dups, dec.t_place, t_wait,
                         (pipe || dense_fuse) ? dec.t_recs : dec.t_p2 - dec.t_fields - dec.t_place);
    }
    // the pending chunk's placement finished, its records written, the buffers it read released
    bool drain(const Cols& c) {
        if (!pending) return true;
        const double t0 = now_s();
        placer.wait();
        t_wait += now_s() - t0;
        pending = false;
        if (pend.over) return fail("stream batch payload overflow"), false;
        dec.records_stage(pend, c);
        st.release_held();
        return true;
    }
};

int64_t mgp_bam_ref_records(mgp_bam* b, int tid) {
    if (!b || tid < 0 || tid >= (int)b->ref_names.size() || !b->has_index) return -1;
    return b->ref_records[(size_t)tid];
}

int mgp_bam_stream_open(mgp_bam* b, int tid, int rec_align, mgp_bam_stream** out) {
    g_err.clear();
    if (!b || !out) return fail("null argument");
    if (tid < 0 || tid >= (int)b->ref_names.size()) return fail("reference id out of range");
    if (rec_align < 16 || rec_align > 4096 || (rec_align & (rec_align - 1))) return fail("bad rec_align");
    std::unique_ptr<mgp_bam_stream> s(new (std::nothrow) mgp_bam_stream(b, rec_align));
    if (!s) return fail("out of host memory");
    s->tid = tid;
    uint64_t voff = b->first_record_voff;
    if (b->has_index) {
        voff = b->ref_first_voff[(size_t)tid];
        if (voff == UINT64_MAX) s->done = true;  // no reads on this reference
    }
    const char* ew = std::getenv("MGP_BAM_WALK_AHEAD");
    if (!s->done && !stream_at(b, voff, s->st, !ew || std::strtol(ew, nullptr, 10) != 0)) return -1;
    *out = s.release();
    return 0;
}

int64_t mgp_bam_stream_next(mgp_bam_stream* s, int64_t cap_reads, int64_t cap_payload, mgp_bam_batch* into) {
    g_err.clear();
    if (!s || !into || !into->start || !into->bc || !into->tlen || !into->flag || !into->mapq || !into->span ||
        !into->rec_off || !into->payload)
        return fail("null argument");
    Decoder& dec = s->dec;
    const uint64_t slack = dec.line_slack() + 256;
    if (cap_reads < 1 || cap_payload < (int64_t)(slack + 65536))
        return fail("stream batch capacity too small (payload needs >= 64 KiB + 256 B per cell)");
    const Cols c{into->start, into->bc, into->tlen, into->flag, into->mapq, into->span, into->rec_off, into->payload};
    auto reserve = [&](size_t kn, uint64_t pay_end) {
        return kn <= (size_t)cap_reads && pay_end + 256 <= (uint64_t)cap_payload;
    };
    auto cols = [&]() { return c; };
    // an error return leaves no placement running on the caller's batch arrays
    struct Settle {
        mgp_bam_stream* s;
        ~Settle() {
            if (s->pending) {
                s->placer.wait();
                s->pending = false;
            }
        }
    } settle{s};
    dec.begin_batch();
    std::vector<size_t>& offs = s->offs;
    size_t k = 0;
    uint64_t bound = 0;
    bool full = false;
    Stream& st = s->st;
    while (!s->done && !full && k < (size_t)cap_reads) {
        const double tf0 = now_s();
        if (!st.fill(4)) {
            if (!g_err.empty()) return -1;
            if (st.avail() == 0) {  // clean end of file
                s->done = true;
                break;
            }
            return fail("truncated BAM record");
        }
        const uint32_t bs0 = rd32(st.peek());
        if (bs0 < 32) return fail("corrupt BAM record (block_size < 32)");
        if (!st.fill(4 + (size_t)bs0)) return fail(g_err.empty() ? "truncated BAM record body" : g_err);
        const double tp1 = now_s();
        s->t_fill += tp1 - tf0;
        dec.clear_chunk();
        const uint8_t* base = st.base;
        size_t p = st.pos;
        const size_t end = st.size;
        bool at_end = false;
        offs.clear();
        // record boundaries (the prefetch thread's walk, or sequential here), then pass 1
        // on the pool, then the batch's cut
        // the prefetch walk's list: the carried record (at 0) one by one, then, once the
        // reads are on tid, whole runs of tid's records taken with bulk copies
        bool listed = st.walked;
        const double tl0 = now_s();
        if (listed && p == 0 && st.wt > 0 && end >= 8) {  // the carried record
            const uint32_t bs = rd32(base);
            const int32_t ref = rdi32(base + 4);
            if (end >= 4 + (size_t)bs) {
                if (ref == s->tid) {
                    s->seen = true;
                    dec.recs.push_back(base + 4);
                    dec.sizes.push_back(bs);
                    offs.push_back(0);
                    p = 4 + (size_t)bs;
                } else if (s->seen || ref > s->tid || ref < 0) {
                    at_end = true;
                }
            }
            if (!s->seen) listed = false;  // (still before tid: the walk below finds it)
        }
        size_t wi = 0;
        const std::vector<uint32_t>* rs = nullptr;
        if (listed && !at_end) {
            rs = &st.wc->rstart;
            const size_t rel = p - st.wt;
            wi = (size_t)(std::lower_bound(rs->begin(), rs->end(), (uint32_t)rel) - rs->begin());
            // the chain and the position agree, and the reads are on tid already
            listed = p >= st.wt && s->seen && (wi == rs->size() ? p == end || end - p < 4 : (*rs)[wi] == rel);
        }
        if (listed && !at_end && rs) {
            const Chunk& ch = *st.wc;
            const size_t nw = rs->size();
            size_t i1 = std::min(nw, wi + ((size_t)cap_reads - k - dec.recs.size()));
            // a record that ends past the buffer (the last one) waits for the next chunk
            if (i1 > wi && st.wt + ch.rstart[i1 - 1] + 4 + (size_t)ch.rsize[i1 - 1] > end) --i1;
            // (tid's records are contiguous: a run that starts and ends on tid is all tid
            // when a branch-free pass finds no other reference in it; else the scan)
            size_t j = wi;
            if (i1 > wi && ch.rref[wi] == s->tid && ch.rref[i1 - 1] == s->tid) {
                uint32_t other = 0;
                for (size_t x = wi; x < i1; ++x) other |= (uint32_t)(ch.rref[x] != s->tid);
                if (!other) j = i1;
            }
            while (j < i1 && ch.rref[j] == s->tid) ++j;
            const size_t n0 = dec.recs.size(), cnt = j - wi;
            dec.recs.resize(n0 + cnt);
            dec.sizes.resize(n0 + cnt);
            offs.resize(n0 + cnt);
            // the chunk's record list (a consumer-side pass of ~4 ns per record at C4 on one
            // thread: on the pool for large runs)
            const size_t wt = st.wt;
            auto list = [&, wt, n0, wi](size_t a, size_t b) {
                for (size_t x = a; x < b; ++x) {
                    const size_t q = wt + ch.rstart[wi + x];
                    dec.recs[n0 + x] = base + q + 4;
                    offs[n0 + x] = q;
                }
                std::memcpy(dec.sizes.data() + n0 + a, ch.rsize.data() + wi + a, (b - a) * sizeof(uint32_t));
            };
            const int lt = (int)std::min<size_t>((size_t)dec.pool.size(), cnt / 32768 + 1);
            if (lt > 1)
                dec.pool.run(lt, [&](int t) { list(cnt * (size_t)t / (size_t)lt, cnt * (size_t)(t + 1) / (size_t)lt); });
            else
                list(0, cnt);
            if (cnt) p = offs[n0 + cnt - 1] + 4 + (size_t)ch.rsize[j - 1];
            if (j < i1) at_end = true;  // a record of another reference: tid's records are contiguous
        }
        s->t_list += now_s() - tl0;
        ++(listed ? s->n_listed : s->n_walked);
        while (!listed && !at_end && end - p >= 4 && k + dec.recs.size() < (size_t)cap_reads) {
            // the walk is a chain of dependent header loads over bytes other threads just
            // inflated: keep lines ahead of it in flight
            __builtin_prefetch(base + p + 1024);
            __builtin_prefetch(base + p + 2048);
            const uint32_t bs = rd32(base + p);
            if (bs < 32) return fail("corrupt BAM record (block_size < 32)");
            if (end - p < 4 + (size_t)bs) break;
            const int32_t ref = rdi32(base + p + 4);
            if (ref == s->tid) {
                s->seen = true;
                dec.recs.push_back(base + p + 4);
                dec.sizes.push_back(bs);
                offs.push_back(p);
            } else if (s->seen || ref > s->tid || ref < 0) {
                at_end = true;  // coordinate-sorted: tid's records are contiguous
                break;
            }
            p += 4 + (size_t)bs;
        }
        const double tw = now_s();
        s->t_walk += tw - tp1;
        // pipelined: pass 1 and the columns in one pool pass (one trip through the records'
        // memory; a record cut off below is decoded again with the next batch)
        bool all64 = false;
        if (s->dense_fuse ? !dec.classify_fields_records_all(k, s->decoded + (int64_t)k, c, (uint64_t)cap_payload, all64)
            : s->fuse    ? !dec.classify_fields_all(k, s->decoded + (int64_t)k, c)
                         : !dec.classify_all())
            return -1;
        s->t_class += now_s() - tw;
        for (size_t i = 0; i < dec.recs.size(); ++i) {
            const uint64_t w = dec.worst(i);
            if (bound + w + slack > (uint64_t)cap_payload) {  // the rest goes to the next batch
                p = offs[i];
                dec.truncate(i);
                full = true;
                at_end = false;
                break;
            }
            bound += w;
        }
        if (at_end) s->done = true;
        dec.t_p1 += now_s() - tp1;
        if (!dec.recs.empty()) {
            const size_t m = dec.recs.size();
            if (s->pipe) {
                if (s->fuse) dec.count_tags(s->decoded + (int64_t)k);
                else dec.fields_stage(k, s->decoded + (int64_t)k, c);
                if (!s->drain(c)) return -1;  // the chunk before: placed meanwhile, now its records
                dec.dup_stage(k, c);          // (behind the chunk before's placement: cells in order)
                dec.move_chunk(s->pend, k);
                s->pending = true;
                s->placer.submit([s, c, cap_payload] { s->dec.place_stage(s->pend, c, (uint64_t)cap_payload); });
            } else if (s->dense_fuse) {
                dec.count_tags(s->decoded + (int64_t)k);
                if (all64) {  // every record already at cursor + 64 x i
                    for (size_t i = 0; i < m; ++i) c.roff[k + i] = dec.cursor + 64ull * i;
                    dec.cursor += 64ull * m;
                } else {
                    dec.dense_offsets(k, c);
                    dec.records_inline(k, c);
                }
            } else if (dec.decode(k, s->decoded + (int64_t)k, reserve, cols) != 0) {
                return -1;
            }
            k += m;
        }
        st.pos = p;
    }
    if (!s->drain(c)) return -1;
    if (k == 0 && !s->done && full) return fail("stream batch capacity too small for one record");
    // >= 256 bytes of zeroed slack after the payload (kernels read up to 128 past a record)
    std::memset(into->payload + dec.cursor, 0, std::min<uint64_t>(256, (uint64_t)cap_payload - dec.cursor));
    into->n_reads = (int64_t)k;
    into->payload_bytes = (int64_t)dec.cursor;
    into->n_with_tag = dec.n_tag;
    into->first_tag_index = dec.first_tag;
    s->decoded += (int64_t)k;
    return (int64_t)k;
}

void mgp_bam_stream_close(mgp_bam_stream* s) { delete s; }

void mgp_bam_free_batch(mgp_bam_batch* x) {
    if (!x) return;
    std::free(x->start);
    std::free(x->bc);
    std::free(x->tlen);
    std::free(x->flag);
    std::free(x->mapq);
    std::free(x->span);
    std::free(x->rec_off);
    std::free(x->payload);
    std::memset(x, 0, sizeof(*x));
}

int64_t mgp_bam_find_tag(mgp_bam* b, int tid, const char* tag, int64_t max_records, int64_t* n_checked) {
    g_err.clear();
    if (!b || !tag || std::strlen(tag) != 2) return fail("bad arguments");
    if (tid < 0 || tid >= (int)b->ref_names.size()) return fail("reference id out of range");
    char tg[3] = {tag[0], tag[1], 0};
    int64_t i = 0, found = -1;
    const int rc = for_each_record(b, tid, [&](const uint8_t* r, uint32_t bs) -> int {
        if (i >= max_records) return 0;
        const uint8_t l_name = r[8];
        const uint32_t n_cig = rd16(r + 12);
        const uint32_t l_seq = rd32(r + 16);
        const uint8_t* auxp = r + 32 + l_name + 4 * (size_t)n_cig + ((size_t)l_seq + 1) / 2 + l_seq;
        if (auxp > r + bs) return fail("corrupt BAM record (fields exceed block_size)"), -1;
        Aux aux{auxp, r + bs};
        if (aux.find(tg)) {
            found = i;
            return 0;
        }
        ++i;
        return 1;
    });
    if (rc != 0) return -2;
    if (n_checked) *n_checked = found >= 0 ? found + 1 : i;
    return found;
}

int64_t mgp_bam_count_tag(mgp_bam* b, int tid, const char* tag, uint8_t** blob, int64_t* blob_bytes) {
    g_err.clear();
    if (!b || !tag || std::strlen(tag) != 2 || !blob || !blob_bytes) return fail("bad arguments");
    if (tid < 0 || tid >= (int)b->ref_names.size()) return fail("reference id out of range");
    std::unordered_map<std::string, int64_t> counts;
    std::vector<std::string> order;
    char tg[3] = {tag[0], tag[1], 0};
    const int rc = for_each_record(b, tid, [&](const uint8_t* r, uint32_t bs) -> int {
        const uint16_t flg = rd16(r + 14);
        if (flg & (0x4 | 0x400)) return 1;  // is_unmapped or is_duplicate (barcode_extraction.py:26)
        const uint8_t l_name = r[8];
        const uint32_t n_cig = rd16(r + 12);
        const uint32_t l_seq = rd32(r + 16);
        const uint8_t* auxp = r + 32 + l_name + 4 * (size_t)n_cig + ((size_t)l_seq + 1) / 2 + l_seq;
        Aux aux{auxp, r + bs};
        const uint8_t* t = aux.find(tg);
        if (!t) return 1;
        std::string v;
        switch (t[0]) {  // str(read.get_tag(tag))
            case 'Z': case 'H': v = (const char*)t + 1; break;
            case 'A': v = std::string(1, (char)t[1]); break;
            case 'c': v = std::to_string((int8_t)t[1]); break;
            case 'C': v = std::to_string((uint8_t)t[1]); break;
            case 's': v = std::to_string((int16_t)rd16(t + 1)); break;
            case 'S': v = std::to_string(rd16(t + 1)); break;
            case 'i': v = std::to_string(rdi32(t + 1)); break;
            case 'I': v = std::to_string(rd32(t + 1)); break;
            default: return 1;  // float / array tags are not barcodes
        }
        auto it = counts.find(v);
        if (it == counts.end()) {
            counts.emplace(v, 1);
            order.push_back(v);
        } else {
            ++it->second;
        }
        return 1;
    });
    if (rc != 0) return -1;
    size_t bytes = 0;
    for (const auto& k : order) bytes += k.size() + 1 + 8;
    uint8_t* p = (uint8_t*)std::malloc(std::max<size_t>(bytes, 1));
    if (!p) return fail("out of host memory");
    size_t o = 0;
    for (const auto& k : order) {
        std::memcpy(p + o, k.c_str(), k.size() + 1);
        o += k.size() + 1;
        const int64_t c = counts[k];
        std::memcpy(p + o, &c, 8);
        o += 8;
    }
    *blob = p;
    *blob_bytes = (int64_t)bytes;
    return (int64_t)order.size();
}

}  // extern "C"
