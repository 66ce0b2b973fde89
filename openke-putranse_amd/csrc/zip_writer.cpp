// Checkpoint archive writer (host only): the zip container torch.save produces (stored records, 64-byte aligned
// data, ZIP64 when a size, an offset or the record count needs it), written from plain memory with the GIL released
// (ctypes) and the CRC-32s computed in parallel (zlib crc32_z per slice, joined with crc32_combine). A CRC the
// caller already knows (an immutable record written before) is reused: the caller keeps what this call returns.
// Used by openke/config/_checkpoint.py for Parallel_Universe_Config.save_parameters (:890-899).
#include <zlib.h>

#include <algorithm>
#include <cerrno>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "putranse.h"

namespace {

constexpr uint64_t k32 = 0xFFFFFFFFull;

uint32_t crc_parallel(const uint8_t *p, int64_t n, int threads) {
    const int64_t slice = int64_t(8) << 20;
    const int parts = static_cast<int>(std::min<int64_t>(std::max(threads, 1), (n + slice - 1) / slice));
    if (parts <= 1) return static_cast<uint32_t>(crc32_z(0L, p, static_cast<z_size_t>(n)));
    std::vector<uLong> crc(parts);
    std::vector<int64_t> lo(parts + 1);
    for (int i = 0; i <= parts; ++i) lo[i] = n * i / parts;
    std::vector<std::thread> pool;
    for (int i = 0; i < parts; ++i)
        pool.emplace_back([&, i] { crc[i] = crc32_z(0L, p + lo[i], static_cast<z_size_t>(lo[i + 1] - lo[i])); });
    for (auto &t : pool) t.join();
    uLong c = crc[0];
    for (int i = 1; i < parts; ++i) c = crc32_combine64(c, crc[i], static_cast<z_off64_t>(lo[i + 1] - lo[i]));
    return static_cast<uint32_t>(c);
}

struct Out {
    std::string buf;
    void u16(uint32_t v) { buf.push_back(char(v & 0xff)); buf.push_back(char((v >> 8) & 0xff)); }
    void u32(uint64_t v) { for (int i = 0; i < 4; ++i) buf.push_back(char((v >> (8 * i)) & 0xff)); }
    void u64(uint64_t v) { for (int i = 0; i < 8; ++i) buf.push_back(char((v >> (8 * i)) & 0xff)); }
    void bytes(const void *p, size_t n) { buf.append(static_cast<const char *>(p), n); }
};

bool write_all(FILE *f, const void *p, size_t n) { return n == 0 || std::fwrite(p, 1, n, f) == n; }

}  // namespace

extern "C" int pt_zip_write(const char *path, pt_zip_record *recs, int64_t n, int32_t alignment, int32_t threads,
                            int32_t force_zip64) {
    if (!path || n < 0 || (n && !recs) || alignment <= 0 || (alignment & (alignment - 1))) return PT_EINVAL;
    for (int64_t i = 0; i < n; ++i) {
        if (!recs[i].name || recs[i].size < 0 || (recs[i].size && !recs[i].data)) return PT_EINVAL;
        if (std::strlen(recs[i].name) >= 0xFFFF) return PT_EINVAL;
    }
    for (int64_t i = 0; i < n; ++i)
        if (!recs[i].crc_known) {
            recs[i].crc32 = crc_parallel(static_cast<const uint8_t *>(recs[i].data), recs[i].size, threads);
            recs[i].crc_known = 1;
        }
    FILE *f = std::fopen(path, "wb");
    if (!f) return PT_EIO;
    std::vector<uint64_t> offset(n);
    std::vector<char> pad(alignment + 4, 'Z');
    uint64_t pos = 0;
    bool ok = true;
    for (int64_t i = 0; i < n && ok; ++i) {
        const pt_zip_record &r = recs[i];
        const size_t name_len = std::strlen(r.name);
        const uint64_t size = static_cast<uint64_t>(r.size);
        const bool z64 = force_zip64 || size >= k32;
        offset[i] = pos;
        const uint64_t base = pos + 30 + name_len + (z64 ? 20 : 0);
        // 'FB' padding field (as torch's writer): the record data starts on an `alignment` boundary
        const uint64_t pad_len = (alignment - (base + 4) % alignment) % alignment;
        Out h;
        h.u32(0x04034b50);
        h.u16(z64 ? 45 : 20);   // version needed
        h.u16(0);               // flags
        h.u16(0);               // stored
        h.u16(0);
        h.u16(0);               // time, date
        h.u32(r.crc32);
        h.u32(z64 ? k32 : size);
        h.u32(z64 ? k32 : size);
        h.u16(static_cast<uint32_t>(name_len));
        h.u16(static_cast<uint32_t>((z64 ? 20 : 0) + 4 + pad_len));
        h.bytes(r.name, name_len);
        if (z64) {
            h.u16(0x0001);
            h.u16(16);
            h.u64(size);
            h.u64(size);
        }
        h.u16(0x4246);
        h.u16(static_cast<uint32_t>(pad_len));
        h.bytes(pad.data(), pad_len);
        ok = write_all(f, h.buf.data(), h.buf.size()) && write_all(f, r.data, size);
        pos += h.buf.size() + size;
    }
    const uint64_t cd_off = pos;
    Out cd;
    bool any64 = force_zip64 != 0;
    for (int64_t i = 0; i < n; ++i) {
        const pt_zip_record &r = recs[i];
        const size_t name_len = std::strlen(r.name);
        const uint64_t size = static_cast<uint64_t>(r.size);
        const bool big = force_zip64 || size >= k32, far = force_zip64 || offset[i] >= k32;
        any64 = any64 || big || far;
        const uint32_t ext = (big ? 16 : 0) + (far ? 8 : 0);
        cd.u32(0x02014b50);
        cd.u16(45);                   // version made by
        cd.u16(big || far ? 45 : 20);
        cd.u16(0);
        cd.u16(0);
        cd.u16(0);
        cd.u16(0);
        cd.u32(r.crc32);
        cd.u32(big ? k32 : size);
        cd.u32(big ? k32 : size);
        cd.u16(static_cast<uint32_t>(name_len));
        cd.u16(ext ? ext + 4 : 0);
        cd.u16(0);                    // comment
        cd.u16(0);                    // disk
        cd.u16(0);                    // internal attributes
        cd.u32(0);                    // external attributes
        cd.u32(far ? k32 : offset[i]);
        cd.bytes(r.name, name_len);
        if (ext) {
            cd.u16(0x0001);
            cd.u16(ext);
            if (big) {
                cd.u64(size);
                cd.u64(size);
            }
            if (far) cd.u64(offset[i]);
        }
    }
    const uint64_t cd_size = cd.buf.size();
    any64 = any64 || n >= 0xFFFF || cd_off >= k32 || cd_size >= k32;
    Out end;
    if (any64) {
        const uint64_t z64_off = cd_off + cd_size;
        end.u32(0x06064b50);
        end.u64(44);
        end.u16(45);
        end.u16(45);
        end.u32(0);
        end.u32(0);
        end.u64(static_cast<uint64_t>(n));
        end.u64(static_cast<uint64_t>(n));
        end.u64(cd_size);
        end.u64(cd_off);
        end.u32(0x07064b50);
        end.u32(0);
        end.u64(z64_off);
        end.u32(1);
    }
    end.u32(0x06054b50);
    end.u16(0);
    end.u16(0);
    end.u16(any64 ? 0xFFFF : static_cast<uint32_t>(n));
    end.u16(any64 ? 0xFFFF : static_cast<uint32_t>(n));
    end.u32(any64 ? k32 : cd_size);
    end.u32(any64 ? k32 : cd_off);
    end.u16(0);
    ok = ok && write_all(f, cd.buf.data(), cd.buf.size()) && write_all(f, end.buf.data(), end.buf.size());
    ok = (std::fclose(f) == 0) && ok;
    return ok ? PT_OK : PT_EIO;
}
