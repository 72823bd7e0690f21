// TF1 "V2" checkpoint (tensor bundle) reader/writer without TensorFlow.
//
// <prefix>.index : a LevelDB-format SSTable.  Keys are tensor names (sorted, the empty key
//                  holds the BundleHeaderProto), values are serialized BundleEntryProto
//                  {dtype=1, shape=2, shard_id=3, offset=4, size=5, crc32c=6 (fixed32)}.
//                  Blocks: prefix-compressed entries + restart array, each followed by a
//                  5-byte trailer {compression=0, masked crc32c}; footer = metaindex handle
//                  + index handle (varints, padded to 40 B) + magic 0xdb4775248b80fb57.
// <prefix>.data-00000-of-00001 : raw little-endian tensor bytes back to back.
//
// Masked CRC32C (Castagnoli) everywhere, as TF/LevelDB: ((c >> 15) | (c << 17)) + 0xa282ead8.
// Exposed as a plain C ABI for ctypes (textsummarization_on_flink_amd/runtime/tf_bundle.py).
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <map>
#include <string>
#include <vector>

namespace {

uint32_t crc_table[256];
struct CrcInit {
  CrcInit() {
    for (uint32_t i = 0; i < 256; ++i) {
      uint32_t c = i;
      for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ 0x82F63B78u : (c >> 1);
      crc_table[i] = c;
    }
  }
} crc_init_;

uint32_t crc32c_extend(uint32_t crc, const uint8_t* p, size_t n) {
  crc = ~crc;
  for (size_t i = 0; i < n; ++i) crc = crc_table[(crc ^ p[i]) & 0xff] ^ (crc >> 8);
  return ~crc;
}
uint32_t mask(uint32_t c) { return ((c >> 15) | (c << 17)) + 0xa282ead8u; }
uint32_t unmask(uint32_t m) {
  uint32_t r = m - 0xa282ead8u;
  return (r >> 17) | (r << 15);
}

void put_varint(std::string& s, uint64_t v) {
  while (v >= 0x80) {
    s.push_back(char((v & 0x7f) | 0x80));
    v >>= 7;
  }
  s.push_back(char(v));
}
bool get_varint(const uint8_t*& p, const uint8_t* end, uint64_t& v) {
  v = 0;
  for (int shift = 0; shift < 64 && p < end; shift += 7) {
    uint8_t b = *p++;
    v |= uint64_t(b & 0x7f) << shift;
    if (!(b & 0x80)) return true;
  }
  return false;
}
void put_fixed32(std::string& s, uint32_t v) { for (int i = 0; i < 4; ++i) s.push_back(char((v >> (8 * i)) & 0xff)); }
void put_fixed64(std::string& s, uint64_t v) { for (int i = 0; i < 8; ++i) s.push_back(char((v >> (8 * i)) & 0xff)); }
uint32_t get_fixed32(const uint8_t* p) { return p[0] | (p[1] << 8) | (p[2] << 16) | (uint32_t(p[3]) << 24); }
uint64_t get_fixed64(const uint8_t* p) { return uint64_t(get_fixed32(p)) | (uint64_t(get_fixed32(p + 4)) << 32); }
void put_tag(std::string& s, int field, int wt) { put_varint(s, (uint64_t(field) << 3) | wt); }
void put_bytes(std::string& s, int field, const std::string& b) { put_tag(s, field, 2); put_varint(s, b.size()); s += b; }

const uint64_t kMagic = 0xdb4775248b80fb57ull;

struct Entry {
  int dtype = 0;
  std::vector<int64_t> shape;
  int shard = 0;
  int64_t offset = 0, size = 0;
  uint32_t crc = 0;  // masked
};

std::string encode_entry(const Entry& e) {
  std::string s, shp;
  put_tag(s, 1, 0); put_varint(s, e.dtype);
  for (int64_t d : e.shape) {
    std::string dim;
    put_tag(dim, 1, 0); put_varint(dim, uint64_t(d));
    put_bytes(shp, 2, dim);
  }
  put_bytes(s, 2, shp);
  if (e.shard) { put_tag(s, 3, 0); put_varint(s, e.shard); }
  if (e.offset) { put_tag(s, 4, 0); put_varint(s, uint64_t(e.offset)); }
  if (e.size) { put_tag(s, 5, 0); put_varint(s, uint64_t(e.size)); }
  put_tag(s, 6, 5); put_fixed32(s, e.crc);
  return s;
}

bool decode_entry(const uint8_t* p, const uint8_t* end, Entry& e) {
  while (p < end) {
    uint64_t key;
    if (!get_varint(p, end, key)) return false;
    int f = int(key >> 3), wt = int(key & 7);
    uint64_t v = 0;
    if (wt == 0) {
      if (!get_varint(p, end, v)) return false;
      if (f == 1) e.dtype = int(v);
      else if (f == 3) e.shard = int(v);
      else if (f == 4) e.offset = int64_t(v);
      else if (f == 5) e.size = int64_t(v);
    } else if (wt == 5) {
      if (end - p < 4) return false;
      if (f == 6) e.crc = get_fixed32(p);
      p += 4;
    } else if (wt == 1) {
      p += 8;
    } else if (wt == 2) {
      if (!get_varint(p, end, v) || uint64_t(end - p) < v) return false;
      const uint8_t* q = p;
      const uint8_t* qe = p + v;
      if (f == 2) {  // TensorShapeProto
        while (q < qe) {
          uint64_t k2, len;
          if (!get_varint(q, qe, k2)) return false;
          if ((k2 & 7) == 2) {
            if (!get_varint(q, qe, len)) return false;
            if ((k2 >> 3) == 2) {  // Dim
              const uint8_t* r = q;
              const uint8_t* re = q + len;
              int64_t size = 0;
              while (r < re) {
                uint64_t k3, x;
                if (!get_varint(r, re, k3)) return false;
                if ((k3 & 7) == 0) { if (!get_varint(r, re, x)) return false; if ((k3 >> 3) == 1) size = int64_t(x); }
                else if ((k3 & 7) == 2) { if (!get_varint(r, re, x)) return false; r += x; }
                else return false;
              }
              e.shape.push_back(size);
            }
            q += len;
          } else if ((k2 & 7) == 0) {
            uint64_t x;
            if (!get_varint(q, qe, x)) return false;
          } else return false;
        }
      }
      p += v;
    } else {
      return false;
    }
  }
  return true;
}

// ----------------------------------------------------------------- SSTable writer
struct BlockBuilder {
  std::string buf;
  std::vector<uint32_t> restarts{0};
  std::string last;
  int counter = 0;
  void add(const std::string& k, const std::string& v) {
    size_t shared = 0;
    if (counter < 16) {
      size_t m = std::min(last.size(), k.size());
      while (shared < m && last[shared] == k[shared]) ++shared;
    } else {
      restarts.push_back(uint32_t(buf.size()));
      counter = 0;
    }
    put_varint(buf, shared);
    put_varint(buf, k.size() - shared);
    put_varint(buf, v.size());
    buf.append(k, shared, std::string::npos);
    buf += v;
    last = k;
    ++counter;
  }
  std::string finish() {
    std::string out = buf;
    for (uint32_t r : restarts) put_fixed32(out, r);
    put_fixed32(out, uint32_t(restarts.size()));
    return out;
  }
  bool empty() const { return buf.empty(); }
};

void write_block(std::string& file, const std::string& contents, uint64_t& off, uint64_t& size) {
  off = file.size();
  size = contents.size();
  file += contents;
  std::string trailer(1, '\0');
  uint32_t c = crc32c_extend(0, reinterpret_cast<const uint8_t*>(contents.data()), contents.size());
  c = crc32c_extend(c, reinterpret_cast<const uint8_t*>(trailer.data()), 1);
  put_fixed32(trailer, mask(c));
  file += trailer;
}

struct Writer {
  std::string prefix;
  std::map<std::string, Entry> entries;
  std::FILE* data = nullptr;
  int64_t off = 0;
};

struct Reader {
  std::string prefix;
  std::vector<std::string> names;
  std::vector<Entry> entries;
  std::FILE* data = nullptr;
  std::string err;
};

bool read_file(const std::string& path, std::string& out) {
  std::ifstream f(path, std::ios::binary);
  if (!f) return false;
  out.assign(std::istreambuf_iterator<char>(f), std::istreambuf_iterator<char>());
  return true;
}

bool parse_block(const std::string& file, uint64_t off, uint64_t size, bool verify,
                 std::vector<std::pair<std::string, std::string>>& kv) {
  if (off + size + 5 > file.size()) return false;
  const uint8_t* b = reinterpret_cast<const uint8_t*>(file.data()) + off;
  if (verify) {
    uint32_t c = crc32c_extend(0, b, size + 1);
    if (unmask(get_fixed32(b + size + 1)) != c) return false;
  }
  if (b[size] != 0) return false;  // compressed blocks are not produced by TF bundles
  if (size < 4) return false;
  uint32_t nrest = get_fixed32(b + size - 4);
  if (size < 4 + 4ull * nrest) return false;
  const uint8_t* p = b;
  const uint8_t* end = b + size - 4 - 4 * nrest;
  std::string key;
  while (p < end) {
    uint64_t shared, nons, vlen;
    if (!get_varint(p, end, shared) || !get_varint(p, end, nons) || !get_varint(p, end, vlen)) return false;
    if (shared > key.size() || uint64_t(end - p) < nons + vlen) return false;
    key.resize(shared);
    key.append(reinterpret_cast<const char*>(p), nons);
    p += nons;
    kv.emplace_back(key, std::string(reinterpret_cast<const char*>(p), vlen));
    p += vlen;
  }
  return true;
}

}  // namespace

extern "C" {

uint32_t tsb_crc32c(const void* data, uint64_t n) { return crc32c_extend(0, static_cast<const uint8_t*>(data), n); }
uint32_t tsb_crc32c_masked(const void* data, uint64_t n) { return mask(tsb_crc32c(data, n)); }

void* tsb_writer_open(const char* prefix) {
  auto* w = new Writer;
  w->prefix = prefix;
  std::string dp = w->prefix + ".data-00000-of-00001";
  w->data = std::fopen(dp.c_str(), "wb");
  if (!w->data) { delete w; return nullptr; }
  return w;
}

// dtype: TF DataType enum (DT_FLOAT=1, DT_DOUBLE=2, DT_INT32=3, DT_INT64=9, DT_BFLOAT16=14, DT_HALF=19)
int tsb_writer_add(void* h, const char* name, int dtype, int ndims, const int64_t* dims, const void* bytes,
                   int64_t nbytes) {
  auto* w = static_cast<Writer*>(h);
  if (!w || !name || !*name || w->entries.count(name)) return -1;
  Entry e;
  e.dtype = dtype;
  e.shape.assign(dims, dims + ndims);
  e.offset = w->off;
  e.size = nbytes;
  e.crc = mask(crc32c_extend(0, static_cast<const uint8_t*>(bytes), size_t(nbytes)));
  if (nbytes && std::fwrite(bytes, 1, size_t(nbytes), w->data) != size_t(nbytes)) return -2;
  w->off += nbytes;
  w->entries[name] = e;
  return 0;
}

int tsb_writer_finish(void* h) {
  auto* w = static_cast<Writer*>(h);
  if (!w) return -1;
  int rc = std::fclose(w->data) == 0 ? 0 : -2;
  std::string file;
  std::vector<std::pair<std::string, std::pair<uint64_t, uint64_t>>> index;
  BlockBuilder bb;
  // header entry under the empty key: BundleHeaderProto{num_shards=1, endianness=LITTLE, version{producer=1}}
  std::string hdr, ver;
  put_tag(hdr, 1, 0); put_varint(hdr, 1);
  put_tag(ver, 1, 0); put_varint(ver, 1);
  put_bytes(hdr, 3, ver);
  std::vector<std::pair<std::string, std::string>> kvs;
  kvs.emplace_back("", hdr);
  for (auto& it : w->entries) kvs.emplace_back(it.first, encode_entry(it.second));
  for (auto& kv : kvs) {
    bb.add(kv.first, kv.second);
    if (bb.buf.size() >= 262144) {
      uint64_t o, s;
      write_block(file, bb.finish(), o, s);
      index.push_back({bb.last, {o, s}});
      bb = BlockBuilder();
    }
  }
  if (!bb.empty()) {
    uint64_t o, s;
    write_block(file, bb.finish(), o, s);
    index.push_back({bb.last, {o, s}});
  }
  uint64_t mo, ms, io, is;
  write_block(file, BlockBuilder().finish(), mo, ms);  // empty meta-index
  BlockBuilder ib;
  for (auto& e : index) {
    std::string hv;
    put_varint(hv, e.second.first);
    put_varint(hv, e.second.second);
    ib.add(e.first, hv);
  }
  write_block(file, ib.finish(), io, is);
  std::string footer;
  put_varint(footer, mo); put_varint(footer, ms);
  put_varint(footer, io); put_varint(footer, is);
  footer.resize(40, '\0');
  put_fixed64(footer, kMagic);
  file += footer;
  std::string ip = w->prefix + ".index";
  std::FILE* f = std::fopen(ip.c_str(), "wb");
  if (!f) { delete w; return -3; }
  if (std::fwrite(file.data(), 1, file.size(), f) != file.size()) rc = -4;
  std::fclose(f);
  delete w;
  return rc;
}

void* tsb_reader_open(const char* prefix, int verify) {
  auto* r = new Reader;
  r->prefix = prefix;
  std::string file;
  if (!read_file(r->prefix + ".index", file) || file.size() < 48) { delete r; return nullptr; }
  const uint8_t* ft = reinterpret_cast<const uint8_t*>(file.data()) + file.size() - 48;
  if (get_fixed64(ft + 40) != kMagic) { delete r; return nullptr; }
  uint64_t mo, ms, io, is;
  const uint8_t* p = ft;
  const uint8_t* pe = ft + 40;
  if (!get_varint(p, pe, mo) || !get_varint(p, pe, ms) || !get_varint(p, pe, io) || !get_varint(p, pe, is)) {
    delete r; return nullptr;
  }
  std::vector<std::pair<std::string, std::string>> idx;
  if (!parse_block(file, io, is, verify, idx)) { delete r; return nullptr; }
  for (auto& e : idx) {
    const uint8_t* q = reinterpret_cast<const uint8_t*>(e.second.data());
    const uint8_t* qe = q + e.second.size();
    uint64_t bo, bs;
    if (!get_varint(q, qe, bo) || !get_varint(q, qe, bs)) { delete r; return nullptr; }
    std::vector<std::pair<std::string, std::string>> kv;
    if (!parse_block(file, bo, bs, verify, kv)) { delete r; return nullptr; }
    for (auto& x : kv) {
      if (x.first.empty()) continue;  // header
      Entry en;
      const uint8_t* a = reinterpret_cast<const uint8_t*>(x.second.data());
      if (!decode_entry(a, a + x.second.size(), en)) { delete r; return nullptr; }
      r->names.push_back(x.first);
      r->entries.push_back(en);
    }
  }
  std::string dp = r->prefix + ".data-00000-of-00001";
  r->data = std::fopen(dp.c_str(), "rb");
  if (!r->data) { delete r; return nullptr; }
  return r;
}

int tsb_reader_num(void* h) { return h ? int(static_cast<Reader*>(h)->names.size()) : -1; }

// Fills name (nul-terminated, up to name_cap), dtype, ndims, dims (up to 8), nbytes.
int tsb_reader_entry(void* h, int i, char* name, int name_cap, int* dtype, int* ndims, int64_t* dims, int64_t* nbytes) {
  auto* r = static_cast<Reader*>(h);
  if (!r || i < 0 || i >= int(r->names.size())) return -1;
  const std::string& n = r->names[i];
  if (int(n.size()) + 1 > name_cap) return -2;
  std::memcpy(name, n.c_str(), n.size() + 1);
  const Entry& e = r->entries[i];
  *dtype = e.dtype;
  *ndims = int(e.shape.size());
  for (size_t k = 0; k < e.shape.size() && k < 8; ++k) dims[k] = e.shape[k];
  *nbytes = e.size;
  return 0;
}

// Reads tensor i into out (nbytes); returns 0, -3 on I/O error, -4 on crc mismatch.
int tsb_reader_read(void* h, int i, void* out, int verify) {
  auto* r = static_cast<Reader*>(h);
  if (!r || i < 0 || i >= int(r->names.size())) return -1;
  const Entry& e = r->entries[i];
  if (e.shard != 0) return -5;
  if (std::fseek(r->data, long(e.offset), SEEK_SET) != 0) return -3;
  if (e.size && std::fread(out, 1, size_t(e.size), r->data) != size_t(e.size)) return -3;
  if (verify && mask(crc32c_extend(0, static_cast<const uint8_t*>(out), size_t(e.size))) != e.crc) return -4;
  return 0;
}

void tsb_reader_close(void* h) {
  auto* r = static_cast<Reader*>(h);
  if (!r) return;
  if (r->data) std::fclose(r->data);
  delete r;
}

}  // extern "C"
