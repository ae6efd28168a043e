// pt_tfrecord.cpp — native GZIP TFRecord reader / writer for PathTracker clips.
//
// Replaces the reference's tf.data pipeline (utils/TFRDataset.py:6-53): files
// are decompressed and parsed by a pool of decoder threads (one file at a
// time per thread, several files in flight), records are handed out in file
// order, optionally through a tf.data-style shuffle buffer, and copied into
// caller-owned batch buffers.  See include/pt_tfrecord.h.
#include "../../include/pt_tfrecord.h"

#include <dlfcn.h>
#include <zlib.h>

#include <algorithm>
#include <condition_variable>
#include <deque>
#include <memory>
#include <mutex>
#include <stdio.h>
#include <string.h>
#include <string>
#include <thread>
#include <vector>

namespace {

thread_local char g_err[512];
template <class... A>
int fail(int code, const char* fmt, A... a) {
  snprintf(g_err, sizeof(g_err), fmt, a...);
  return code;
}

// ---------------------------------------------------------------- CRC32C
// Castagnoli polynomial (reflected 0x82F63B78), slicing-by-8 tables.
struct Crc32cTables {
  uint32_t t[8][256];
  Crc32cTables() {
    for (uint32_t i = 0; i < 256; ++i) {
      uint32_t c = i;
      for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ 0x82F63B78u : c >> 1;
      t[0][i] = c;
    }
    for (int s = 1; s < 8; ++s)
      for (uint32_t i = 0; i < 256; ++i) t[s][i] = (t[s - 1][i] >> 8) ^ t[0][t[s - 1][i] & 0xff];
  }
};
const Crc32cTables& crc_tables() {
  static const Crc32cTables tb;
  return tb;
}
// SSE4.2 crc32 instruction (same polynomial), 8 bytes per step; picked at
// run time so the library still loads on hosts without it.
__attribute__((target("sse4.2"))) uint32_t crc32c_hw(const uint8_t* p, size_t n) {
  uint64_t c = 0xFFFFFFFFu;
  while (n >= 8) {
    uint64_t v;
    memcpy(&v, p, 8);
    c = __builtin_ia32_crc32di(c, v);
    p += 8;
    n -= 8;
  }
  uint32_t c32 = (uint32_t)c;
  while (n--) c32 = __builtin_ia32_crc32qi(c32, *p++);
  return c32 ^ 0xFFFFFFFFu;
}
const bool kHwCrc = __builtin_cpu_supports("sse4.2");
uint32_t crc32c(const uint8_t* p, size_t n) {
  if (kHwCrc) return crc32c_hw(p, n);
  const auto& T = crc_tables().t;
  uint32_t c = 0xFFFFFFFFu;
  while (n >= 8) {
    uint32_t lo, hi;
    memcpy(&lo, p, 4);
    memcpy(&hi, p + 4, 4);
    lo ^= c;
    c = T[7][lo & 0xff] ^ T[6][(lo >> 8) & 0xff] ^ T[5][(lo >> 16) & 0xff] ^ T[4][lo >> 24] ^
        T[3][hi & 0xff] ^ T[2][(hi >> 8) & 0xff] ^ T[1][(hi >> 16) & 0xff] ^ T[0][hi >> 24];
    p += 8;
    n -= 8;
  }
  while (n--) c = (c >> 8) ^ T[0][(c ^ *p++) & 0xff];
  return c ^ 0xFFFFFFFFu;
}
uint32_t masked(uint32_t c) { return ((c >> 15) | (c << 17)) + 0xa282ead8u; }

// ------------------------------------------------------- protobuf (wire)
// Minimal decoder for tf.train.Example (tensorflow/core/example/example.proto,
// feature.proto): Example{1: Features}, Features{1: map<string, Feature>},
// entry{1: key, 2: Feature}, Feature{1: BytesList, 2: FloatList, 3: Int64List},
// BytesList{1: repeated bytes}.  Unknown fields are skipped by wire type.
struct Span {
  const uint8_t* p;
  size_t n;
};

bool varint(const uint8_t*& p, const uint8_t* e, uint64_t& v) {
  v = 0;
  for (int s = 0; s < 64 && p < e; s += 7) {
    const uint8_t b = *p++;
    v |= (uint64_t)(b & 0x7f) << s;
    if (!(b & 0x80)) return true;
  }
  return false;
}

// Iterate the fields of a message; f(field, wiretype, span-or-varint).
template <class F>
bool fields(Span m, F&& f) {
  const uint8_t *p = m.p, *e = m.p + m.n;
  while (p < e) {
    uint64_t tag;
    if (!varint(p, e, tag)) return false;
    const int fld = (int)(tag >> 3), wt = (int)(tag & 7);
    uint64_t v = 0;
    Span s{nullptr, 0};
    switch (wt) {
      case 0:
        if (!varint(p, e, v)) return false;
        break;
      case 1:
        if (e - p < 8) return false;
        p += 8;
        break;
      case 2: {
        uint64_t len;
        if (!varint(p, e, len) || (uint64_t)(e - p) < len) return false;
        s = Span{p, (size_t)len};
        p += len;
        break;
      }
      case 5:
        if (e - p < 4) return false;
        p += 4;
        break;
      default:
        return false;
    }
    if (!f(fld, wt, s, v)) return false;
  }
  return true;
}

// 'image' and 'label' bytes of one Example (first value of each BytesList).
bool parse_example(Span ex, Span& image, Span& label, bool& has_image, bool& has_label) {
  has_image = has_label = false;
  return fields(ex, [&](int f, int wt, Span s, uint64_t) {
    if (f != 1 || wt != 2) return true;                       // Example.features
    return fields(s, [&](int f2, int wt2, Span entry, uint64_t) {
      if (f2 != 1 || wt2 != 2) return true;                   // Features.feature (map entry)
      Span key{nullptr, 0}, val{nullptr, 0};
      if (!fields(entry, [&](int f3, int wt3, Span x, uint64_t) {
            if (wt3 == 2 && f3 == 1) key = x;
            if (wt3 == 2 && f3 == 2) val = x;
            return true;
          }))
        return false;
      const bool is_img = key.n == 5 && !memcmp(key.p, "image", 5);
      const bool is_lab = key.n == 5 && !memcmp(key.p, "label", 5);
      if (!is_img && !is_lab) return true;
      return fields(val, [&](int f4, int wt4, Span bl, uint64_t) {
        if (f4 != 1 || wt4 != 2) return true;                 // Feature.bytes_list
        bool first = true;
        return fields(bl, [&](int f5, int wt5, Span b, uint64_t) {
          if (f5 == 1 && wt5 == 2 && first) {
            first = false;
            if (is_img) { image = b; has_image = true; }
            else { label = b; has_label = true; }
          }
          return true;
        });
      });
    });
  });
}

// ------------------------------------------------------- protobuf (write)
void put_varint(std::string& o, uint64_t v) {
  while (v >= 0x80) {
    o.push_back((char)(v | 0x80));
    v >>= 7;
  }
  o.push_back((char)v);
}
void put_len(std::string& o, int field, const std::string& payload) {
  put_varint(o, ((uint64_t)field << 3) | 2);
  put_varint(o, payload.size());
  o += payload;
}
std::string feature_bytes(const uint8_t* p, size_t n) {
  std::string bl, f;
  put_len(bl, 1, std::string((const char*)p, n));   // BytesList.value
  put_len(f, 1, bl);                                 // Feature.bytes_list
  return f;
}
std::string feature_int64(int64_t v) {
  std::string il, f;
  std::string packed;
  put_varint(packed, (uint64_t)v);
  put_len(il, 1, packed);                            // Int64List.value (packed)
  put_len(f, 3, il);                                 // Feature.int64_list
  return f;
}
std::string map_entry(const char* key, const std::string& feat) {
  std::string e;
  put_len(e, 1, key);
  put_len(e, 2, feat);
  return e;
}
// keys in sorted order (deterministic serialisation)
std::string encode_example(const uint8_t* img, size_t nimg, uint8_t label, int64_t h, int64_t w) {
  std::string feats, ex;
  put_len(feats, 1, map_entry("height", feature_int64(h)));
  put_len(feats, 1, map_entry("image", feature_bytes(img, nimg)));
  put_len(feats, 1, map_entry("label", feature_bytes(&label, 1)));
  put_len(feats, 1, map_entry("width", feature_int64(w)));
  put_len(ex, 1, feats);
  return ex;
}

// ------------------------------------------------------------ file reading
// A decompressed file, shared by the records that point into it (records of
// several files mix in the shuffle buffer; the buffer dies with its last one).
struct FileBuf {
  std::vector<uint8_t> raw;
};
struct Clip {
  std::shared_ptr<const FileBuf> buf;
  const uint8_t* img = nullptr;        // into buf->raw, T*H*W*C bytes
  uint8_t label = 0;
};

struct FileResult {
  std::vector<Clip> clips;
  int err = 0;
  std::string msg;
  bool done = false;
};

// ---------------------------------------------------- libdeflate fast path
// The system's libdeflate (runtime library only, no header in the image) is
// ~2-3x faster than zlib at inflating whole gzip members; resolved with dlopen
// at first use, zlib is the fallback.  Its stable C API (libdeflate.h):
struct libdeflate_decompressor;
typedef libdeflate_decompressor* (*ld_alloc_t)(void);
typedef int (*ld_gzip_ex_t)(libdeflate_decompressor*, const void* in, size_t in_nbytes, void* out,
                            size_t out_nbytes_avail, size_t* actual_in_nbytes_ret,
                            size_t* actual_out_nbytes_ret);
typedef void (*ld_free_t)(libdeflate_decompressor*);
struct LibDeflate {
  ld_alloc_t alloc = nullptr;
  ld_gzip_ex_t gzip_ex = nullptr;
  ld_free_t free_ = nullptr;
  LibDeflate() {
    const char* off = getenv("PT_TFR_ZLIB_ONLY");
    if (off && atoi(off)) return;
    void* h = dlopen("libdeflate.so.0", RTLD_NOW | RTLD_LOCAL);
    if (!h) return;
    alloc = (ld_alloc_t)dlsym(h, "libdeflate_alloc_decompressor");
    gzip_ex = (ld_gzip_ex_t)dlsym(h, "libdeflate_gzip_decompress_ex");
    free_ = (ld_free_t)dlsym(h, "libdeflate_free_decompressor");
    if (!alloc || !gzip_ex || !free_) alloc = nullptr;
  }
  bool ok() const { return alloc != nullptr; }
};
const LibDeflate& libdeflate() {
  static const LibDeflate ld;
  return ld;
}

// Whole file -> memory; gzip members inflated by libdeflate.  Returns 1 if the
// fast path is unavailable (caller falls back to zlib), 0 on success, < 0 on error.
int read_all_libdeflate(const std::string& path, std::vector<uint8_t>& out, std::string& msg) {
  const LibDeflate& ld = libdeflate();
  if (!ld.ok()) return 1;
  FILE* fp = fopen(path.c_str(), "rb");
  if (!fp) {
    msg = "cannot open " + path;
    return PT_TFR_ERR_IO;
  }
  std::vector<uint8_t> in;
  if (fseek(fp, 0, SEEK_END) == 0) {
    const long sz = ftell(fp);
    if (sz > 0) in.resize((size_t)sz);
    fseek(fp, 0, SEEK_SET);
  }
  const size_t got = in.empty() ? 0 : fread(in.data(), 1, in.size(), fp);
  fclose(fp);
  if (got != in.size()) {
    msg = "short read on " + path;
    return PT_TFR_ERR_IO;
  }
  if (in.size() < 18 || in[0] != 0x1f || in[1] != 0x8b) {      // not gzip: the file as is
    out.swap(in);
    return 0;
  }
  libdeflate_decompressor* d = ld.alloc();
  if (!d) return 1;
  // output estimate: the last member's ISIZE, grown on demand
  const uint8_t* t = in.data() + in.size() - 4;
  size_t cap = (size_t)t[0] | ((size_t)t[1] << 8) | ((size_t)t[2] << 16) | ((size_t)t[3] << 24);
  if (cap < (1u << 20)) cap = 1u << 20;
  out.resize(cap);
  size_t ipos = 0, opos = 0;
  int rc = 0;
  while (ipos < in.size()) {                   // concatenated members
    size_t in_used = 0, out_len = 0;
    const int r = ld.gzip_ex(d, in.data() + ipos, in.size() - ipos, out.data() + opos,
                             out.size() - opos, &in_used, &out_len);
    if (r == 3) {                              // LIBDEFLATE_INSUFFICIENT_SPACE
      out.resize(out.size() * 2);
      continue;
    }
    if (r != 0) {
      msg = "gzip error in " + path + " (libdeflate " + std::to_string(r) + ")";
      rc = PT_TFR_ERR_FORMAT;
      break;
    }
    ipos += in_used;
    opos += out_len;
  }
  ld.free_(d);
  if (rc) return rc;
  out.resize(opos);
  return 0;
}

int read_all(const std::string& path, std::vector<uint8_t>& out, std::string& msg) {
  if (int rc = read_all_libdeflate(path, out, msg); rc <= 0) return rc;
  gzFile f = gzopen(path.c_str(), "rb");       // transparently reads plain files too
  if (!f) {
    msg = "cannot open " + path;
    return PT_TFR_ERR_IO;
  }
  gzbuffer(f, 1 << 20);
  // size hint: a single-member gzip stream ends with ISIZE (length mod 2^32)
  size_t cap = 1 << 22;
  if (FILE* fp = fopen(path.c_str(), "rb")) {
    unsigned char tail[4];
    if (fseek(fp, -4, SEEK_END) == 0 && fread(tail, 1, 4, fp) == 4) {
      const size_t isize = tail[0] | (tail[1] << 8) | (tail[2] << 16) | ((size_t)tail[3] << 24);
      if (isize > cap) cap = isize + 1;
    }
    fclose(fp);
  }
  out.resize(cap);
  size_t len = 0;
  for (;;) {
    if (len == out.size()) out.resize(out.size() * 2);
    const size_t want = std::min<size_t>(out.size() - len, 1u << 30);
    const int n = gzread(f, out.data() + len, (unsigned)want);
    if (n < 0) {
      int zerr;
      msg = std::string("gzip error in ") + path + ": " + gzerror(f, &zerr);
      gzclose(f);
      return PT_TFR_ERR_FORMAT;
    }
    if (n == 0) break;
    len += (size_t)n;
  }
  gzclose(f);
  out.resize(len);
  return 0;
}

void decode_file(const std::string& path, const pt_tfr_options& o, FileResult& r) {
  auto fb = std::make_shared<FileBuf>();
  if (int rc = read_all(path, fb->raw, r.msg)) { r.err = rc; return; }
  const std::vector<uint8_t>& raw = fb->raw;
  const size_t need = (size_t)o.timesteps * o.height * o.width * o.channels;
  size_t off = 0;
  int64_t rec = 0;
  char m[256];
  while (off < raw.size()) {
    if (raw.size() - off < 12) {
      snprintf(m, sizeof(m), "%s: truncated record header at byte %zu", path.c_str(), off);
      r.msg = m; r.err = PT_TFR_ERR_FORMAT; return;
    }
    uint64_t len;
    uint32_t lcrc;
    memcpy(&len, raw.data() + off, 8);
    memcpy(&lcrc, raw.data() + off + 8, 4);
    if (o.verify_crc && masked(crc32c(raw.data() + off, 8)) != lcrc) {
      snprintf(m, sizeof(m), "%s: record %lld length CRC mismatch", path.c_str(), (long long)rec);
      r.msg = m; r.err = PT_TFR_ERR_FORMAT; return;
    }
    // no `len + 4`: a corrupt length near UINT64_MAX would wrap and pass
    const uint64_t avail = raw.size() - off - 12;
    if (len > avail || avail - len < 4) {
      snprintf(m, sizeof(m), "%s: truncated record %lld", path.c_str(), (long long)rec);
      r.msg = m; r.err = PT_TFR_ERR_FORMAT; return;
    }
    const uint8_t* data = raw.data() + off + 12;
    uint32_t dcrc;
    memcpy(&dcrc, data + len, 4);
    if (o.verify_crc && masked(crc32c(data, len)) != dcrc) {
      snprintf(m, sizeof(m), "%s: record %lld data CRC mismatch", path.c_str(), (long long)rec);
      r.msg = m; r.err = PT_TFR_ERR_FORMAT; return;
    }
    Span img{nullptr, 0}, lab{nullptr, 0};
    bool hi, hl;
    if (!parse_example(Span{data, (size_t)len}, img, lab, hi, hl) || !hi || !hl) {
      snprintf(m, sizeof(m), "%s: record %lld is not an Example with 'image' and 'label' bytes",
               path.c_str(), (long long)rec);
      r.msg = m; r.err = PT_TFR_ERR_FORMAT; return;
    }
    if (img.n != need) {       // tf.reshape([T, 32, 32, 3]) fails on any other size
      snprintf(m, sizeof(m), "%s: record %lld image has %zu bytes, expected %zu", path.c_str(),
               (long long)rec, img.n, need);
      r.msg = m; r.err = PT_TFR_ERR_FORMAT; return;
    }
    if (lab.n != 1) {          // engine.prepare_data ord()s the label: one byte only
      snprintf(m, sizeof(m), "%s: record %lld label has %zu bytes, expected 1", path.c_str(),
               (long long)rec, lab.n);
      r.msg = m; r.err = PT_TFR_ERR_FORMAT; return;
    }
    Clip c;
    c.buf = fb;
    c.img = img.p;
    c.label = lab.p[0];
    r.clips.push_back(std::move(c));
    off += 12 + len + 4;
    ++rec;
  }
}

}  // namespace

// ------------------------------------------------------------------ reader
struct pt_tfr_reader {
  pt_tfr_options o;
  std::vector<std::string> files;              // this rank's files, in order
  std::vector<std::unique_ptr<FileResult>> res;
  size_t next_submit = 0, next_consume = 0, pos_in_file = 0;
  std::mutex mu;
  std::condition_variable cv;
  std::vector<std::thread> pool;
  std::deque<size_t> queue;                    // file indices waiting for a thread
  bool stop = false;
  // shuffle buffer
  std::vector<Clip> buf;
  uint64_t rng;
  int64_t produced = 0;
  bool exhausted = false;

  uint64_t next_rand() {                       // splitmix64
    uint64_t z = (rng += 0x9e3779b97f4a7c15ull);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
  }

  void worker() {
    for (;;) {
      size_t fi;
      {
        std::unique_lock<std::mutex> lk(mu);
        cv.wait(lk, [&] { return stop || !queue.empty(); });
        if (stop) return;
        fi = queue.front();
        queue.pop_front();
      }
      FileResult tmp;
      decode_file(files[fi], o, tmp);
      {
        std::lock_guard<std::mutex> lk(mu);
        res[fi]->clips = std::move(tmp.clips);
        res[fi]->err = tmp.err;
        res[fi]->msg = std::move(tmp.msg);
        res[fi]->done = true;
      }
      cv.notify_all();
    }
  }

  // keep up to threads + 1 files decoded or in flight ahead of the consumer
  void submit_ahead() {
    std::lock_guard<std::mutex> lk(mu);
    const size_t ahead = (size_t)o.threads + 1;
    while (next_submit < files.size() && next_submit < next_consume + ahead) {
      queue.push_back(next_submit++);
    }
    cv.notify_all();
  }

  // next record in file order; false at the end; err on failure
  bool next_record(Clip& out, int& err) {
    err = 0;
    while (next_consume < files.size()) {
      submit_ahead();
      FileResult* r = res[next_consume].get();
      {
        std::unique_lock<std::mutex> lk(mu);
        cv.wait(lk, [&] { return r->done; });
      }
      if (r->err) {
        snprintf(g_err, sizeof(g_err), "%s", r->msg.c_str());
        err = r->err;
        return false;
      }
      if (pos_in_file < r->clips.size()) {
        out = std::move(r->clips[pos_in_file++]);
        return true;
      }
      r->clips.clear();
      r->clips.shrink_to_fit();
      ++next_consume;
      pos_in_file = 0;
    }
    return false;
  }

  // tf.data shuffle(buffer): fill the buffer, then each output is a uniformly
  // chosen slot, refilled from the input stream.
  bool next_sample(Clip& out, int& err) {
    err = 0;
    if (o.shuffle_buffer <= 0) return next_record(out, err);
    while (!exhausted && (int)buf.size() < o.shuffle_buffer) {
      Clip c;
      if (!next_record(c, err)) {
        if (err) return false;
        exhausted = true;
        break;
      }
      buf.push_back(std::move(c));
    }
    if (buf.empty()) return false;
    const size_t i = (size_t)(next_rand() % buf.size());
    out = std::move(buf[i]);
    Clip c;
    if (!exhausted && next_record(c, err)) {
      buf[i] = std::move(c);
    } else {
      if (err) return false;
      exhausted = true;
      buf[i] = std::move(buf.back());
      buf.pop_back();
    }
    return true;
  }
};

extern "C" {

uint32_t pt_tfr_crc32c(const uint8_t* data, size_t n) { return crc32c(data, n); }
uint32_t pt_tfr_masked_crc32c(const uint8_t* data, size_t n) { return masked(crc32c(data, n)); }

pt_tfr_reader* pt_tfr_open(const char* const* paths, int32_t npaths, const pt_tfr_options* o) {
  if (!paths || npaths < 0 || !o) { fail(PT_TFR_ERR_ARG, "%s", "null paths / options"); return nullptr; }
  if (o->timesteps < 1 || o->height < 1 || o->width < 1 || o->channels < 1) {
    fail(PT_TFR_ERR_ARG, "%s", "clip shape must be positive");
    return nullptr;
  }
  if (o->world < 1 || o->rank < 0 || o->rank >= o->world) {
    fail(PT_TFR_ERR_ARG, "rank %d outside world %d", o->rank, o->world);
    return nullptr;
  }
  auto* r = new pt_tfr_reader();
  r->o = *o;
  if (r->o.threads < 1) r->o.threads = 1;
  r->rng = o->seed ^ (0x5bd1e995ull * (uint64_t)(o->rank + 1));
  for (int i = 0; i < npaths; ++i)
    if (i % o->world == o->rank) r->files.emplace_back(paths[i]);
  for (size_t i = 0; i < r->files.size(); ++i) r->res.emplace_back(new FileResult());
  for (int i = 0; i < r->o.threads; ++i) r->pool.emplace_back([r] { r->worker(); });
  return r;
}

int64_t pt_tfr_next(pt_tfr_reader* r, int32_t batch, uint8_t* clips, uint8_t* labels) {
  if (!r || batch < 1 || !clips || !labels) return fail(PT_TFR_ERR_ARG, "%s", "bad arguments to pt_tfr_next");
  const size_t need = (size_t)r->o.timesteps * r->o.height * r->o.width * r->o.channels;
  // stage first: with drop_remainder a short batch is discarded, so nothing is
  // written to the caller's buffers unless the batch completes
  std::vector<Clip> got;
  got.reserve(batch);
  for (int i = 0; i < batch; ++i) {
    Clip c;
    int err;
    if (!r->next_sample(c, err)) {
      if (err) return err;
      break;
    }
    got.push_back(std::move(c));
  }
  if (got.empty() || (r->o.drop_remainder && (int)got.size() < batch)) return 0;
  for (size_t i = 0; i < got.size(); ++i) {
    memcpy(clips + i * need, got[i].img, need);
    labels[i] = got[i].label;
  }
  r->produced += (int64_t)got.size();
  return (int64_t)got.size();
}

int64_t pt_tfr_count(const pt_tfr_reader* r) { return r ? r->produced : (int64_t)PT_TFR_ERR_ARG; }

int pt_tfr_close(pt_tfr_reader* r) {
  if (!r) return PT_TFR_ERR_ARG;
  {
    std::lock_guard<std::mutex> lk(r->mu);
    r->stop = true;
  }
  r->cv.notify_all();
  for (auto& t : r->pool) t.join();
  delete r;
  return 0;
}

int pt_tfr_write(const char* path, const uint8_t* clips, const uint8_t* labels, int64_t n, int32_t t,
                 int32_t h, int32_t w, int32_t c, int32_t gzip) {
  if (!path || (n > 0 && (!clips || !labels)) || n < 0 || t < 1 || h < 1 || w < 1 || c < 1)
    return fail(PT_TFR_ERR_ARG, "%s", "bad arguments to pt_tfr_write");
  const size_t need = (size_t)t * h * w * c;
  std::string out;
  for (int64_t i = 0; i < n; ++i) {
    const std::string ex = encode_example(clips + i * need, need, labels[i], h, w);
    const uint64_t len = ex.size();
    uint8_t hdr[12];
    memcpy(hdr, &len, 8);
    const uint32_t lc = masked(crc32c(hdr, 8));
    memcpy(hdr + 8, &lc, 4);
    out.append((const char*)hdr, 12);
    out += ex;
    const uint32_t dc = masked(crc32c((const uint8_t*)ex.data(), ex.size()));
    out.append((const char*)&dc, 4);
  }
  if (gzip) {
    gzFile f = gzopen(path, "wb6");
    if (!f) return fail(PT_TFR_ERR_IO, "cannot open %s for writing", path);
    size_t off = 0;
    while (off < out.size()) {
      const unsigned chunk = (unsigned)std::min<size_t>(out.size() - off, 1u << 30);
      if (gzwrite(f, out.data() + off, chunk) != (int)chunk) {
        gzclose(f);
        return fail(PT_TFR_ERR_IO, "gzwrite failed on %s", path);
      }
      off += chunk;
    }
    if (gzclose(f) != Z_OK) return fail(PT_TFR_ERR_IO, "gzclose failed on %s", path);
  } else {
    FILE* f = fopen(path, "wb");
    if (!f) return fail(PT_TFR_ERR_IO, "cannot open %s for writing", path);
    const size_t wr = fwrite(out.data(), 1, out.size(), f);
    if (fclose(f) != 0 || wr != out.size()) return fail(PT_TFR_ERR_IO, "write failed on %s", path);
  }
  return 0;
}

int64_t pt_tfr_parse_example(const uint8_t* data, size_t n, uint8_t* image, size_t image_cap,
                             uint8_t* label) {
  if (!data || !image || !label) return fail(PT_TFR_ERR_ARG, "%s", "null argument");
  Span img{nullptr, 0}, lab{nullptr, 0};
  bool hi, hl;
  if (!parse_example(Span{data, n}, img, lab, hi, hl) || !hi || !hl)
    return fail(PT_TFR_ERR_FORMAT, "%s", "not an Example with 'image' and 'label' bytes");
  if (lab.n != 1) return fail(PT_TFR_ERR_FORMAT, "label has %zu bytes, expected 1", lab.n);
  if (img.n > image_cap) return fail(PT_TFR_ERR_ARG, "image has %zu bytes, buffer %zu", img.n, image_cap);
  memcpy(image, img.p, img.n);
  *label = lab.p[0];
  return (int64_t)img.n;
}

const char* pt_tfr_last_error(void) { return g_err; }

}  // extern "C"
