// SID input path, host side: read-only LMDB lookup, PNG decode to uint16 and the crop window,
// feeding the device-side conversion in sid.hip.
//
// Reference: NAFNet_base/basicsr/data/sony_sid_lmdb_dataset.py
//   _load_png_uint16 (:38-56): cv2.imdecode(IMREAD_UNCHANGED) -> uint8 promoted by *257 -> 3 channels required
//     -> BGR2RGB, i.e. the PNG's own R, G, B order as uint16;
//   _fetch_png (:150-160): LMDB value by key (basicsr FileClient 'lmdb': txn.get(key.encode('ascii'))) or a file;
//   _maybe_random_crop (:162-192): the [top, top+ps) x [left, left+ps) window of every array.
// cv2 / libpng and the lmdb package are not in this image: the PNG decoder follows the PNG specification (zlib
// stream, per-row filters 0-4, Adam7, bit depths 1-16, palette expansion) and the LMDB reader the on-disk format
// of LMDB 0.9 (64-bit: 16-byte page headers, two meta pages, B+tree of branch / leaf pages, overflow pages for
// large values).  Both are pure host code: no GPU, no allocation visible to the caller (LMDB files are mmapped).
#include <errno.h>
#include <fcntl.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>
#include <zlib.h>

#include <algorithm>
#include <atomic>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/nbp.h"

namespace nbp {
void set_error(const char* fmt, ...);
}

#define SID_REQUIRE(cond, ...)       \
  do {                               \
    if (!(cond)) {                   \
      ::nbp::set_error(__VA_ARGS__); \
      return NBP_ERR_ARG;            \
    }                                \
  } while (0)

namespace {

// ------------------------------------------------------------------------------------------------------ LMDB
constexpr uint16_t P_BRANCH = 0x01, P_LEAF = 0x02, P_OVERFLOW = 0x04, P_META = 0x08;
constexpr uint16_t F_BIGDATA = 0x01, F_SUBDATA = 0x02, F_DUPDATA = 0x04;
constexpr uint32_t MDB_MAGIC = 0xBEEFC0DE;
constexpr uint64_t P_INVALID = ~0ull;
constexpr size_t PAGEHDRSZ = 16, NODESZ = 8;

template <typename T>
T rd(const uint8_t* p) {
  T v;
  memcpy(&v, p, sizeof(T));
  return v;
}

struct Lmdb {
  const uint8_t* map = nullptr;
  size_t size = 0;
  size_t psize = 4096;
  uint64_t root = P_INVALID;
  uint64_t entries = 0;
  uint64_t txnid = 0;

  const uint8_t* page(uint64_t pgno) const {
    if (pgno == P_INVALID || pgno > size / psize || (pgno + 1) * psize > size) return nullptr;
    return map + pgno * psize;
  }
};

std::mutex g_lmdb_mu;
std::vector<Lmdb*> g_lmdb;  // handle = index

// default LMDB key order (mdb_cmp_memn): bytewise, then the shorter key first
int key_cmp(const uint8_t* a, size_t la, const uint8_t* b, size_t lb) {
  const int c = memcmp(a, b, std::min(la, lb));
  if (c) return c;
  return la < lb ? -1 : (la > lb ? 1 : 0);
}

int lmdb_open(const char* path, Lmdb** out) {
  std::string file(path);
  struct stat st;
  SID_REQUIRE(stat(file.c_str(), &st) == 0, "nbp_lmdb_open: %s: %s", path, strerror(errno));
  if (S_ISDIR(st.st_mode)) {  // lmdb.open(path) default subdir=True: <path>/data.mdb
    file += "/data.mdb";
    SID_REQUIRE(stat(file.c_str(), &st) == 0, "nbp_lmdb_open: %s: %s", file.c_str(), strerror(errno));
  }
  SID_REQUIRE(st.st_size >= 2 * 4096, "nbp_lmdb_open: %s is too small for an LMDB environment", file.c_str());
  const int fd = open(file.c_str(), O_RDONLY);
  SID_REQUIRE(fd >= 0, "nbp_lmdb_open: %s: %s", file.c_str(), strerror(errno));
  void* m = mmap(nullptr, (size_t)st.st_size, PROT_READ, MAP_SHARED, fd, 0);
  close(fd);
  SID_REQUIRE(m != MAP_FAILED, "nbp_lmdb_open: mmap %s: %s", file.c_str(), strerror(errno));
  Lmdb* db = new Lmdb;
  db->map = (const uint8_t*)m;
  db->size = (size_t)st.st_size;
  // meta pages 0 and 1 (the page size is recorded in the FREE db's md_pad); the newer valid one wins
  const uint8_t* mp0 = db->map;
  const uint32_t psize = rd<uint32_t>(mp0 + PAGEHDRSZ + 24);
  bool ok = psize >= 512 && psize <= 65536 && (psize & (psize - 1)) == 0 && 2 * (size_t)psize <= db->size;
  int best = -1;
  uint64_t best_txn = 0;
  for (int i = 0; ok && i < 2; ++i) {
    const uint8_t* p = db->map + (size_t)i * psize;
    if (!(rd<uint16_t>(p + 10) & P_META) || rd<uint32_t>(p + PAGEHDRSZ) != MDB_MAGIC) continue;
    const uint64_t txn = rd<uint64_t>(p + PAGEHDRSZ + 24 + 2 * 48 + 8);
    if (best < 0 || txn > best_txn) best = i, best_txn = txn;
  }
  if (!ok || best < 0) {
    munmap(m, db->size);
    delete db;
    SID_REQUIRE(false, "nbp_lmdb_open: %s is not an LMDB data file (no valid meta page)", file.c_str());
  }
  const uint8_t* meta = db->map + (size_t)best * psize + PAGEHDRSZ;
  const uint8_t* main_db = meta + 24 + 48;  // mm_dbs[MAIN_DBI]
  const uint16_t version = (uint16_t)rd<uint32_t>(meta + 4);
  db->psize = psize;
  db->entries = rd<uint64_t>(main_db + 32);
  db->root = rd<uint64_t>(main_db + 40);
  db->txnid = best_txn;
  if (version != 1 || (rd<uint16_t>(main_db + 4) & 0x04 /* MDB_DUPSORT */)) {
    munmap(m, db->size);
    delete db;
    SID_REQUIRE(false, "nbp_lmdb_open: %s: unsupported LMDB format (version %u, or a DUPSORT main db)",
                file.c_str(), version);
  }
  *out = db;
  return 0;
}

// key lookup: 1 found (value pointer into the map), 0 not found, < 0 corrupt
int lmdb_get(const Lmdb* db, const uint8_t* key, size_t klen, const uint8_t** val, size_t* vlen) {
  uint64_t pgno = db->root;
  if (pgno == P_INVALID) return 0;
  for (int depth = 0; depth < 64; ++depth) {
    const uint8_t* p = db->page(pgno);
    SID_REQUIRE(p, "nbp_lmdb_get: page %llu out of range", (unsigned long long)pgno);
    const uint16_t flags = rd<uint16_t>(p + 10), lower = rd<uint16_t>(p + 12);
    SID_REQUIRE(lower >= PAGEHDRSZ && lower <= db->psize, "nbp_lmdb_get: corrupt page %llu", (unsigned long long)pgno);
    const int n = (lower - (int)PAGEHDRSZ) >> 1;
    auto node = [&](int i, const uint8_t** k, size_t* kl) -> const uint8_t* {
      const uint16_t off = rd<uint16_t>(p + PAGEHDRSZ + 2 * i);
      if (off + NODESZ > db->psize) return nullptr;
      const uint8_t* nd = p + off;
      *kl = rd<uint16_t>(nd + 6);
      *k = nd + NODESZ;
      if (off + NODESZ + *kl > db->psize) return nullptr;
      return nd;
    };
    if (flags & P_BRANCH) {
      SID_REQUIRE(n >= 1, "nbp_lmdb_get: empty branch page");
      // child i covers [key_i, key_{i+1}); key_0 is implicitly the lowest
      int lo = 1, hi = n - 1, pick = 0;
      while (lo <= hi) {
        const int mid = (lo + hi) / 2;
        const uint8_t* k;
        size_t kl;
        SID_REQUIRE(node(mid, &k, &kl), "nbp_lmdb_get: corrupt branch node");
        if (key_cmp(key, klen, k, kl) >= 0) pick = mid, lo = mid + 1;
        else hi = mid - 1;
      }
      const uint8_t* k;
      size_t kl;
      const uint8_t* nd = node(pick, &k, &kl);
      SID_REQUIRE(nd, "nbp_lmdb_get: corrupt branch node");
      pgno = (uint64_t)rd<uint16_t>(nd) | ((uint64_t)rd<uint16_t>(nd + 2) << 16) |
             ((uint64_t)rd<uint16_t>(nd + 4) << 32);
      continue;
    }
    SID_REQUIRE(flags & P_LEAF, "nbp_lmdb_get: page %llu is neither branch nor leaf", (unsigned long long)pgno);
    int lo = 0, hi = n - 1;
    while (lo <= hi) {
      const int mid = (lo + hi) / 2;
      const uint8_t* k;
      size_t kl;
      const uint8_t* nd = node(mid, &k, &kl);
      SID_REQUIRE(nd, "nbp_lmdb_get: corrupt leaf node");
      const int c = key_cmp(key, klen, k, kl);
      if (c < 0) { hi = mid - 1; continue; }
      if (c > 0) { lo = mid + 1; continue; }
      const uint16_t nf = rd<uint16_t>(nd + 4);
      SID_REQUIRE(!(nf & (F_SUBDATA | F_DUPDATA)), "nbp_lmdb_get: sub-database / duplicate values unsupported");
      const size_t dsz = (size_t)rd<uint16_t>(nd) | ((size_t)rd<uint16_t>(nd + 2) << 16);
      const uint8_t* data = k + kl;
      if (nf & F_BIGDATA) {
        SID_REQUIRE(data + 8 <= p + db->psize, "nbp_lmdb_get: corrupt overflow reference");
        const uint64_t opg = rd<uint64_t>(data);
        const uint8_t* op = db->page(opg);
        SID_REQUIRE(op && (rd<uint16_t>(op + 10) & P_OVERFLOW), "nbp_lmdb_get: bad overflow page");
        const uint32_t npages = rd<uint32_t>(op + 12);
        SID_REQUIRE(PAGEHDRSZ + dsz <= (size_t)npages * db->psize && (opg + npages) * db->psize <= db->size,
                    "nbp_lmdb_get: overflow value exceeds the file");
        *val = op + PAGEHDRSZ;
      } else {
        SID_REQUIRE(data + dsz <= p + db->psize, "nbp_lmdb_get: corrupt inline value");
        *val = data;
      }
      *vlen = dsz;
      return 1;
    }
    return 0;
  }
  SID_REQUIRE(false, "nbp_lmdb_get: tree deeper than 64 levels (corrupt)");
  return NBP_ERR_INTERNAL;
}

// ------------------------------------------------------------------------------------------------------ PNG
struct PngInfo {
  int w = 0, h = 0, depth = 0, ctype = 0, interlace = 0;
  int channels = 0;  // samples per pixel in the file
  bool trns = false;
  std::vector<uint8_t> plte;
  struct Chunk {
    const uint8_t* data;
    size_t n;
    uint32_t crc;
  };
  std::vector<Chunk> idat;  // CRCs checked as each chunk is consumed (a cropped decode stops early)
};

uint32_t be32(const uint8_t* p) { return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3]; }

// header_only: stop at the first IDAT (IHDR / PLTE / tRNS are all before it)
int png_parse(const uint8_t* buf, size_t len, PngInfo* pi, bool header_only = false) {
  static const uint8_t sig[8] = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1a, '\n'};
  SID_REQUIRE(buf && len >= 8 && memcmp(buf, sig, 8) == 0, "PNG: bad signature");
  size_t pos = 8;
  bool ihdr = false, iend = false;
  while (pos + 12 <= len && !iend) {
    const uint32_t n = be32(buf + pos);
    const uint8_t* type = buf + pos + 4;
    SID_REQUIRE(n <= len && pos + 12 + n <= len, "PNG: truncated chunk");
    const uint8_t* data = buf + pos + 8;
    const uint32_t crc = be32(data + n);
    const bool is_idat = !memcmp(type, "IDAT", 4);
    if (is_idat && header_only) break;
    // libpng's default: a CRC error in a critical chunk is an error, in an ancillary chunk it is discarded
    const bool critical = !(type[0] & 0x20);
    SID_REQUIRE(is_idat || !critical || crc32(crc32(0, nullptr, 0), type, n + 4) == crc,
                "PNG: CRC mismatch in chunk %.4s", (const char*)type);
    if (!memcmp(type, "IHDR", 4)) {
      SID_REQUIRE(n == 13 && !ihdr, "PNG: bad IHDR");
      pi->w = (int)be32(data);
      pi->h = (int)be32(data + 4);
      pi->depth = data[8];
      pi->ctype = data[9];
      pi->interlace = data[12];
      SID_REQUIRE(data[10] == 0 && data[11] == 0 && pi->interlace <= 1, "PNG: unknown compression/filter/interlace");
      SID_REQUIRE(pi->w > 0 && pi->h > 0 && pi->w <= (1 << 24) && pi->h <= (1 << 24), "PNG: bad dimensions");
      const int d = pi->depth;
      switch (pi->ctype) {
        case 0: SID_REQUIRE(d == 1 || d == 2 || d == 4 || d == 8 || d == 16, "PNG: bad depth"); pi->channels = 1; break;
        case 2: SID_REQUIRE(d == 8 || d == 16, "PNG: bad depth"); pi->channels = 3; break;
        case 3: SID_REQUIRE(d == 1 || d == 2 || d == 4 || d == 8, "PNG: bad depth"); pi->channels = 1; break;
        case 4: SID_REQUIRE(d == 8 || d == 16, "PNG: bad depth"); pi->channels = 2; break;
        case 6: SID_REQUIRE(d == 8 || d == 16, "PNG: bad depth"); pi->channels = 4; break;
        default: SID_REQUIRE(false, "PNG: bad color type %d", pi->ctype);
      }
      ihdr = true;
    } else if (!memcmp(type, "PLTE", 4)) {
      SID_REQUIRE(n % 3 == 0 && n <= 768, "PNG: bad PLTE");
      pi->plte.assign(data, data + n);
    } else if (!memcmp(type, "tRNS", 4)) {
      pi->trns = true;
    } else if (is_idat) {
      pi->idat.push_back({data, n, crc});
    } else if (!memcmp(type, "IEND", 4)) {
      iend = true;
    } else {
      SID_REQUIRE(type[0] & 0x20, "PNG: unknown critical chunk %.4s", (const char*)type);
    }
    pos += 12 + n;
  }
  SID_REQUIRE(ihdr && (header_only || !pi->idat.empty()), "PNG: missing IHDR or IDAT");
  SID_REQUIRE(pi->ctype != 3 || !pi->plte.empty(), "PNG: palette image without PLTE");
  return 0;
}

// channels of the array cv2.imdecode(IMREAD_UNCHANGED) returns: gray 1; RGB 3; palette 3 (4 with tRNS);
// gray+alpha and RGBA 4
int cv2_channels(const PngInfo& pi) {
  switch (pi.ctype) {
    case 0: return 1;
    case 2: return 3;
    case 3: return pi.trns ? 4 : 3;
    default: return 4;
  }
}

inline uint8_t paeth(int a, int b, int c) {
  const int p = a + b - c, pa = abs(p - a), pb = abs(p - b), pc = abs(p - c);
  return (uint8_t)((pa <= pb && pa <= pc) ? a : (pb <= pc ? b : c));
}

// undo the per-row filter in place; prev = the previous reconstructed row (nullptr for the first)
int unfilter(uint8_t ft, uint8_t* row, const uint8_t* prev, size_t rb, size_t bpp) {
  switch (ft) {
    case 0: break;
    case 1: for (size_t i = bpp; i < rb; ++i) row[i] = (uint8_t)(row[i] + row[i - bpp]); break;
    case 2: if (prev) for (size_t i = 0; i < rb; ++i) row[i] = (uint8_t)(row[i] + prev[i]); break;
    case 3:
      for (size_t i = 0; i < rb; ++i) {
        const int a = i >= bpp ? row[i - bpp] : 0, b = prev ? prev[i] : 0;
        row[i] = (uint8_t)(row[i] + ((a + b) >> 1));
      }
      break;
    case 4:
      for (size_t i = 0; i < rb; ++i) {
        const int a = i >= bpp ? row[i - bpp] : 0, b = prev ? prev[i] : 0, c = (prev && i >= bpp) ? prev[i - bpp] : 0;
        row[i] = (uint8_t)(row[i] + paeth(a, b, c));
      }
      break;
    default: SID_REQUIRE(false, "PNG: bad filter type %d", ft);
  }
  return 0;
}

// sample x of a reconstructed row (any depth), as the raw integer value
inline uint32_t sample(const uint8_t* row, long idx, int depth) {
  if (depth == 16) return (uint32_t)row[2 * idx] << 8 | row[2 * idx + 1];
  if (depth == 8) return row[idx];
  const long bit = idx * depth;
  return (row[bit >> 3] >> (8 - depth - (bit & 7))) & ((1u << depth) - 1);
}

// Decode into out[h][w][3] uint16 (RGB / expanded palette; 8-bit and palette values * 257, i.e. the uint8 -> uint16
// promotion of _load_png_uint16).  Only the 3-channel forms are decoded (the reference rejects the rest).  When
// crop_h > 0, only rows [top, top + crop_h) x columns [left, left + crop_w) are written (out is crop_h x crop_w) and
// inflation stops after the last needed row (non-interlaced images).
int png_decode_rgb16(const uint8_t* buf, size_t len, uint16_t* out, int top, int left, int crop_h, int crop_w) {
  PngInfo pi;
  int rc = png_parse(buf, len, &pi);
  if (rc) return rc;
  SID_REQUIRE(cv2_channels(pi) == 3, "PNG: %d-channel image (3 expected)", cv2_channels(pi));
  const int H = pi.h, W = pi.w, depth = pi.depth, spp = pi.channels;
  if (crop_h <= 0) top = 0, left = 0, crop_h = H, crop_w = W;
  SID_REQUIRE(top >= 0 && left >= 0 && crop_w > 0 && top + crop_h <= H && left + crop_w <= W,
              "PNG: crop window outside the %dx%d image", H, W);
  const size_t bpp = std::max<size_t>(1, (size_t)spp * depth / 8);
  const int ncol = (int)pi.plte.size() / 3;
  auto emit = [&](int y, int x, const uint8_t* row, long idx) -> int {
    if (y < top || y >= top + crop_h || x < left || x >= left + crop_w) return 0;
    uint16_t* o = out + ((size_t)(y - top) * crop_w + (x - left)) * 3;
    if (pi.ctype == 3) {
      const uint32_t c = sample(row, idx, depth);
      SID_REQUIRE((int)c < ncol, "PNG: palette index %u out of range", c);
      for (int k = 0; k < 3; ++k) o[k] = (uint16_t)(pi.plte[3 * c + k] * 257);
    } else {
      for (int k = 0; k < 3; ++k) {
        const uint32_t v = sample(row, 3 * idx + k, depth);
        o[k] = (uint16_t)(depth == 16 ? v : v * 257);
      }
    }
    return 0;
  };

  z_stream zs;
  memset(&zs, 0, sizeof(zs));
  SID_REQUIRE(inflateInit(&zs) == Z_OK, "PNG: inflateInit failed");
  size_t chunk = 0;
  constexpr int kTruncated = -1000, kBadCrc = -1001;  // distinct from the NBP_ERR_* codes of SID_REQUIRE
  auto inflate_exact = [&](uint8_t* dst, size_t n) -> int {
    zs.next_out = dst;
    zs.avail_out = (uInt)n;
    while (zs.avail_out > 0) {
      if (zs.avail_in == 0) {
        if (chunk >= pi.idat.size()) return kTruncated;
        const PngInfo::Chunk& c = pi.idat[chunk++];
        if (crc32(crc32(crc32(0, nullptr, 0), (const Bytef*)"IDAT", 4), c.data, (uInt)c.n) != c.crc) return kBadCrc;
        zs.next_in = const_cast<Bytef*>(c.data);
        zs.avail_in = (uInt)c.n;
        continue;
      }
      const int z = inflate(&zs, Z_NO_FLUSH);
      if (z == Z_STREAM_END && zs.avail_out > 0) return kTruncated;
      if (z != Z_OK && z != Z_STREAM_END) return kTruncated;
    }
    return 0;
  };

  rc = 0;
  if (!pi.interlace) {
    const size_t rb = ((size_t)W * spp * depth + 7) / 8;
    std::vector<uint8_t> a(rb + 1), b(rb + 1);
    uint8_t *cur = a.data(), *prev = nullptr, *spare = b.data();
    for (int y = 0; y < top + crop_h && !rc; ++y) {
      if ((rc = inflate_exact(cur, rb + 1))) break;
      rc = unfilter(cur[0], cur + 1, prev ? prev + 1 : nullptr, rb, bpp);
      if (rc) break;
      if (y >= top)
        for (int x = left; x < left + crop_w && !rc; ++x) rc = emit(y, x, cur + 1, x);
      uint8_t* t = prev ? prev : spare;
      prev = cur;
      cur = t;
    }
  } else {  // Adam7: 7 reduced images, each filtered independently
    static const int xs[7] = {0, 4, 0, 2, 0, 1, 0}, ys[7] = {0, 0, 4, 0, 2, 0, 1};
    static const int dx[7] = {8, 8, 4, 4, 2, 2, 1}, dy[7] = {8, 8, 8, 4, 4, 2, 2};
    for (int pass = 0; pass < 7 && !rc; ++pass) {
      const int pw = (W - xs[pass] + dx[pass] - 1) / dx[pass], ph = (H - ys[pass] + dy[pass] - 1) / dy[pass];
      if (pw <= 0 || ph <= 0) continue;
      const size_t rb = ((size_t)pw * spp * depth + 7) / 8;
      std::vector<uint8_t> a(rb + 1), b(rb + 1);
      uint8_t *cur = a.data(), *prev = nullptr, *spare = b.data();
      for (int r = 0; r < ph && !rc; ++r) {
        if ((rc = inflate_exact(cur, rb + 1))) break;
        rc = unfilter(cur[0], cur + 1, prev ? prev + 1 : nullptr, rb, bpp);
        const int y = ys[pass] + r * dy[pass];
        for (int i = 0; i < pw && !rc; ++i) rc = emit(y, xs[pass] + i * dx[pass], cur + 1, i);
        uint8_t* t = prev ? prev : spare;
        prev = cur;
        cur = t;
      }
    }
  }
  inflateEnd(&zs);
  SID_REQUIRE(rc != kTruncated, "PNG: truncated or corrupt image data");
  SID_REQUIRE(rc != kBadCrc, "PNG: CRC mismatch in an IDAT chunk");
  return rc;
}

}  // namespace

extern "C" {

int nbp_lmdb_open(const char* path) {
  SID_REQUIRE(path, "nbp_lmdb_open: null path");
  Lmdb* db = nullptr;
  const int rc = lmdb_open(path, &db);
  if (rc) return rc;
  std::lock_guard<std::mutex> g(g_lmdb_mu);
  g_lmdb.push_back(db);
  return (int)g_lmdb.size() - 1;
}

static Lmdb* lmdb_handle(int h) {
  std::lock_guard<std::mutex> g(g_lmdb_mu);
  return h >= 0 && h < (int)g_lmdb.size() ? g_lmdb[h] : nullptr;
}

int nbp_lmdb_close(int handle) {
  std::lock_guard<std::mutex> g(g_lmdb_mu);
  SID_REQUIRE(handle >= 0 && handle < (int)g_lmdb.size() && g_lmdb[handle], "nbp_lmdb_close: bad handle %d", handle);
  munmap(const_cast<uint8_t*>(g_lmdb[handle]->map), g_lmdb[handle]->size);
  delete g_lmdb[handle];
  g_lmdb[handle] = nullptr;
  return 0;
}

int nbp_lmdb_stat(int handle, long* entries, long* psize) {
  const Lmdb* db = lmdb_handle(handle);
  SID_REQUIRE(db && entries && psize, "nbp_lmdb_stat: bad handle or output");
  *entries = (long)db->entries;
  *psize = (long)db->psize;
  return 0;
}

int nbp_lmdb_get(int handle, const char* key, int klen, const void** val, long* vlen) {
  const Lmdb* db = lmdb_handle(handle);
  SID_REQUIRE(db && key && klen >= 0 && val && vlen, "nbp_lmdb_get: bad handle or arguments");
  const uint8_t* v = nullptr;
  size_t n = 0;
  const int rc = lmdb_get(db, (const uint8_t*)key, (size_t)klen, &v, &n);
  if (rc < 0) return rc;
  *val = rc ? v : nullptr;
  *vlen = rc ? (long)n : -1;
  return 0;
}

int nbp_png_info(const void* buf, long len, int* h, int* w, int* channels, int* depth) {
  SID_REQUIRE(buf && len > 0 && h && w && channels && depth, "nbp_png_info: bad arguments");
  PngInfo pi;
  const int rc = png_parse((const uint8_t*)buf, (size_t)len, &pi, true);
  if (rc) return rc;
  *h = pi.h;
  *w = pi.w;
  *channels = cv2_channels(pi);
  *depth = pi.ctype == 3 ? 8 : pi.depth;
  return 0;
}

int nbp_png_decode_rgb16(const void* buf, long len, void* out, int top, int left, int crop_h, int crop_w) {
  SID_REQUIRE(buf && len > 0 && out, "nbp_png_decode_rgb16: bad arguments");
  return png_decode_rgb16((const uint8_t*)buf, (size_t)len, (uint16_t*)out, top, left, crop_h, crop_w);
}

int nbp_png_decode_batch(int n, const void* const* bufs, const long* lens, const int* tops, const int* lefts,
                         int crop_h, int crop_w, void* out, int nthreads) {
  SID_REQUIRE(n >= 0 && (n == 0 || (bufs && lens && tops && lefts && out)) && crop_h > 0 && crop_w > 0,
              "nbp_png_decode_batch: bad arguments (a common crop_h x crop_w window is required)");
  const size_t per = (size_t)crop_h * crop_w * 3;
  std::atomic<int> next{0}, first_bad{-1};
  std::string err;
  std::mutex mu;
  auto work = [&]() {
    for (int i; (i = next.fetch_add(1)) < n;) {
      const int rc = png_decode_rgb16((const uint8_t*)bufs[i], (size_t)lens[i], (uint16_t*)out + per * i, tops[i],
                                      lefts[i], crop_h, crop_w);
      if (rc) {
        std::lock_guard<std::mutex> g(mu);
        if (first_bad.load() < 0 || i < first_bad.load()) {
          first_bad = i;
          err = nbp_last_error_string();  // thread-local message of this worker
        }
      }
    }
  };
  const int nt = std::max(1, std::min(nthreads, n));
  std::vector<std::thread> pool;
  for (int t = 1; t < nt; ++t) pool.emplace_back(work);
  work();
  for (auto& t : pool) t.join();
  SID_REQUIRE(first_bad.load() < 0, "nbp_png_decode_batch: image %d: %s", first_bad.load(), err.c_str());
  return 0;
}

}  // extern "C"
