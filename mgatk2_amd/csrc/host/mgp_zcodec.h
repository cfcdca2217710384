// mgp_zcodec.h — deflate codecs of the host side (libmgphost.so): libdeflate when the
// system has it, zlib otherwise.
//
// BGZF inflate (the BAM decoder), gzip members (txt writer) and zlib streams (HDF5
// deflate filter) are the host stages the node's rate depends on. The image ships
// libdeflate.so.0 (no header): it is opened at run time (dlopen) and its five entry
// points are called through the prototypes of its stable public API; where it is
// absent, zlib does the same work (same decompressed bytes; compressed bytes may
// differ, which every consumer of these formats accepts).
#pragma once
#include <dlfcn.h>
#include <zlib.h>

#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <vector>

namespace mgp_host {

struct LibDeflate {
    using alloc_d_t = void* (*)();
    using free_d_t = void (*)(void*);
    using inflate_t = int (*)(void*, const void*, size_t, void*, size_t, size_t*);
    using crc32_t = uint32_t (*)(uint32_t, const void*, size_t);
    using alloc_c_t = void* (*)(int);
    using free_c_t = void (*)(void*);
    using compress_t = size_t (*)(void*, const void*, size_t, void*, size_t);
    using bound_t = size_t (*)(void*, size_t);
    alloc_d_t alloc_d = nullptr;
    free_d_t free_d = nullptr;
    inflate_t inflate = nullptr;
    crc32_t crc32 = nullptr;
    alloc_c_t alloc_c = nullptr;
    free_c_t free_c = nullptr;
    compress_t gzip = nullptr, zlib = nullptr;
    bound_t gzip_bound = nullptr, zlib_bound = nullptr;
    bool ok = false;
    LibDeflate() {
        if (std::getenv("MGP_NO_LIBDEFLATE")) return;  // (A/B: zlib everywhere)
        void* h = dlopen("libdeflate.so.0", RTLD_NOW | RTLD_LOCAL);
        if (!h) h = dlopen("libdeflate.so", RTLD_NOW | RTLD_LOCAL);
        if (!h) return;
        alloc_d = (alloc_d_t)dlsym(h, "libdeflate_alloc_decompressor");
        free_d = (free_d_t)dlsym(h, "libdeflate_free_decompressor");
        inflate = (inflate_t)dlsym(h, "libdeflate_deflate_decompress");
        crc32 = (crc32_t)dlsym(h, "libdeflate_crc32");
        alloc_c = (alloc_c_t)dlsym(h, "libdeflate_alloc_compressor");
        free_c = (free_c_t)dlsym(h, "libdeflate_free_compressor");
        gzip = (compress_t)dlsym(h, "libdeflate_gzip_compress");
        zlib = (compress_t)dlsym(h, "libdeflate_zlib_compress");
        gzip_bound = (bound_t)dlsym(h, "libdeflate_gzip_compress_bound");
        zlib_bound = (bound_t)dlsym(h, "libdeflate_zlib_compress_bound");
        ok = alloc_d && free_d && inflate && crc32 && alloc_c && free_c && gzip && zlib && gzip_bound && zlib_bound;
    }
    static const LibDeflate& get() {
        static const LibDeflate L;
        return L;
    }
};

inline uint32_t crc32_any(uint32_t crc, const uint8_t* p, size_t n) {
    const LibDeflate& L = LibDeflate::get();
    if (L.ok) return L.crc32(crc, p, n);
    return (uint32_t)::crc32(crc, p, (uInt)n);
}

// Raw deflate stream -> exactly `out_n` bytes (one per thread; not thread-safe).
class Inflator {
  public:
    Inflator() {
        const LibDeflate& L = LibDeflate::get();
        if (L.ok) d_ = L.alloc_d();
        if (!d_) {
            std::memset(&zs_, 0, sizeof(zs_));
            zok_ = inflateInit2(&zs_, -15) == Z_OK;
        }
    }
    ~Inflator() {
        if (d_) LibDeflate::get().free_d(d_);
        else if (zok_) inflateEnd(&zs_);
    }
    Inflator(const Inflator&) = delete;
    Inflator& operator=(const Inflator&) = delete;
    bool raw(const uint8_t* in, size_t in_n, uint8_t* out, size_t out_n) {
        if (d_) {
            size_t got = 0;
            if (LibDeflate::get().inflate(d_, in, in_n, out, out_n, &got) != 0) return false;
            return got == out_n;
        }
        if (!zok_ || inflateReset(&zs_) != Z_OK) return false;
        zs_.next_in = const_cast<uint8_t*>(in);
        zs_.avail_in = (uInt)in_n;
        zs_.next_out = out;
        zs_.avail_out = (uInt)out_n;
        const int r = inflate(&zs_, Z_FINISH);
        return r == Z_STREAM_END && zs_.avail_out == 0;
    }

  private:
    void* d_ = nullptr;
    z_stream zs_;
    bool zok_ = false;
};

// gzip member / zlib stream of a buffer at `level` (one per thread).
class Deflator {
  public:
    explicit Deflator(int level) : level_(level) {
        const LibDeflate& L = LibDeflate::get();
        // (level 0, stored blocks: zlib's form)
        if (L.ok && level > 0) c_ = L.alloc_c(level);
    }
    ~Deflator() {
        if (c_) LibDeflate::get().free_c(c_);
    }
    Deflator(const Deflator&) = delete;
    Deflator& operator=(const Deflator&) = delete;
    bool gzip(const uint8_t* src, size_t n, std::vector<uint8_t>& out) { return run(src, n, out, true); }
    bool zlib(const uint8_t* src, size_t n, std::vector<uint8_t>& out) { return run(src, n, out, false); }

  private:
    bool run(const uint8_t* src, size_t n, std::vector<uint8_t>& out, bool gz) {
        if (c_) {
            const LibDeflate& L = LibDeflate::get();
            out.resize((gz ? L.gzip_bound : L.zlib_bound)(c_, n) + 64);
            const size_t m = (gz ? L.gzip : L.zlib)(c_, src, n, out.data(), out.size());
            if (!m) return false;
            out.resize(m);
            return true;
        }
        z_stream zs;
        std::memset(&zs, 0, sizeof(zs));
        if (deflateInit2(&zs, level_, Z_DEFLATED, gz ? 15 + 16 : 15, 8, Z_DEFAULT_STRATEGY) != Z_OK) return false;
        out.resize(deflateBound(&zs, (uLong)n) + 64);
        zs.next_in = const_cast<uint8_t*>(src);
        zs.avail_in = (uInt)n;
        zs.next_out = out.data();
        zs.avail_out = (uInt)out.size();
        const int r = deflate(&zs, Z_FINISH);
        out.resize(out.size() - zs.avail_out);
        deflateEnd(&zs);
        return r == Z_STREAM_END;
    }
    int level_;
    void* c_ = nullptr;
};

}  // namespace mgp_host
