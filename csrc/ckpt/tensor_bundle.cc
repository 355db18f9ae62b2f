// TF-1.x "V2" checkpoint (TensorBundle) writer/reader -- SURVEY §2.5 N9, §5.4.
//
// Files for prefix P:
//   P.data-00000-of-00001   raw little-endian tensor bytes, back to back
//   P.index                 an SSTable (LevelDB table format) mapping
//                             ""          -> BundleHeaderProto {num_shards=1, endianness=LITTLE, version{producer=1}}
//                             tensor name -> BundleEntryProto  {dtype, shape, shard_id, offset, size, crc32c}
//                           keys sorted bytewise; one data block per <= 64 KiB of entries; index block of
//                           BlockHandles; empty metaindex block; 48-byte footer with the table magic.
// Block trailers carry the masked CRC32C of (block contents + compression byte 0), entries carry
// the masked CRC32C of the tensor bytes -- the same checks TF's reader performs.
// TF is not installed here, so byte compatibility is pinned by a golden structure test against
// the format spec (tests/test_checkpoint.py) rather than against TF output ("parity unpinned").
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <fstream>
#include <map>
#include <stdexcept>
#include <string>
#include <vector>

#include "dtg/bundle.h"

namespace dtg {
namespace ckpt {

// ---- CRC32C (Castagnoli), table driven --------------------------------------------------------
static uint32_t g_crc_table[256];
static bool g_crc_init = false;

static void crc_init() {
  if (g_crc_init) return;
  for (uint32_t i = 0; i < 256; ++i) {
    uint32_t c = i;
    for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ 0x82F63B78u : (c >> 1);
    g_crc_table[i] = c;
  }
  g_crc_init = true;
}

uint32_t crc32c_extend(uint32_t crc, const void* data, size_t n) {
  crc_init();
  const uint8_t* p = (const uint8_t*)data;
  crc = ~crc;
  for (size_t i = 0; i < n; ++i) crc = g_crc_table[(crc ^ p[i]) & 0xff] ^ (crc >> 8);
  return ~crc;
}

uint32_t crc32c(const void* data, size_t n) { return crc32c_extend(0, data, n); }

uint32_t crc_mask(uint32_t crc) { return ((crc >> 15) | (crc << 17)) + 0xa282ead8u; }
uint32_t crc_unmask(uint32_t m) {
  const uint32_t r = m - 0xa282ead8u;
  return (r >> 17) | (r << 15);
}

// ---- protobuf wire helpers ---------------------------------------------------------------------
static void put_varint(std::string* s, uint64_t v) {
  while (v >= 0x80) {
    s->push_back((char)(v | 0x80));
    v >>= 7;
  }
  s->push_back((char)v);
}
static void put_fixed32(std::string* s, uint32_t v) { s->append((const char*)&v, 4); }
static void put_fixed64(std::string* s, uint64_t v) { s->append((const char*)&v, 8); }
static void put_tag(std::string* s, int field, int wt) { put_varint(s, ((uint64_t)field << 3) | (uint64_t)wt); }
static void put_len_field(std::string* s, int field, const std::string& payload) {
  put_tag(s, field, 2);
  put_varint(s, payload.size());
  s->append(payload);
}

static bool get_varint(const uint8_t*& p, const uint8_t* end, uint64_t* v) {
  uint64_t r = 0;
  int shift = 0;
  while (p < end && shift <= 63) {
    const uint8_t b = *p++;
    r |= (uint64_t)(b & 0x7f) << shift;
    if (!(b & 0x80)) {
      *v = r;
      return true;
    }
    shift += 7;
  }
  return false;
}

std::string encode_entry(const Entry& e) {
  std::string s;
  put_tag(&s, 1, 0);
  put_varint(&s, (uint64_t)e.dtype);
  std::string shape;
  for (int64_t d : e.shape) {
    std::string dim;
    put_tag(&dim, 1, 0);
    put_varint(&dim, (uint64_t)d);
    put_len_field(&shape, 2, dim);
  }
  put_len_field(&s, 2, shape);  // TensorShapeProto (present even for scalars)
  if (e.shard_id) {
    put_tag(&s, 3, 0);
    put_varint(&s, (uint64_t)e.shard_id);
  }
  if (e.offset) {
    put_tag(&s, 4, 0);
    put_varint(&s, (uint64_t)e.offset);
  }
  if (e.size) {
    put_tag(&s, 5, 0);
    put_varint(&s, (uint64_t)e.size);
  }
  put_tag(&s, 6, 5);
  put_fixed32(&s, e.crc32c);
  return s;
}

static std::string encode_header() {
  std::string s;
  put_tag(&s, 1, 0);
  put_varint(&s, 1);  // num_shards
  // endianness LITTLE = 0 is the default: omitted, like TF
  std::string ver;
  put_tag(&ver, 1, 0);
  put_varint(&ver, 1);  // producer
  put_len_field(&s, 3, ver);
  return s;
}

static void skip_field(const uint8_t*& p, const uint8_t* end, int wt) {
  uint64_t v;
  switch (wt) {
    case 0: get_varint(p, end, &v); break;
    case 1: p += 8; break;
    case 2: get_varint(p, end, &v); p += v; break;
    case 5: p += 4; break;
    default: throw std::runtime_error("bundle: bad wire type");
  }
}

Entry decode_entry(const std::string& s) {
  Entry e;
  const uint8_t* p = (const uint8_t*)s.data();
  const uint8_t* end = p + s.size();
  while (p < end) {
    uint64_t tag;
    if (!get_varint(p, end, &tag)) throw std::runtime_error("bundle: bad entry");
    const int f = (int)(tag >> 3), wt = (int)(tag & 7);
    uint64_t v = 0;
    if (f == 1 && wt == 0) { get_varint(p, end, &v); e.dtype = (int)v; }
    else if (f == 2 && wt == 2) {
      get_varint(p, end, &v);
      const uint8_t* q = p;
      const uint8_t* qe = p + v;
      while (q < qe) {
        uint64_t t2;
        get_varint(q, qe, &t2);
        if ((t2 >> 3) == 2 && (t2 & 7) == 2) {
          uint64_t dl;
          get_varint(q, qe, &dl);
          const uint8_t* r = q;
          const uint8_t* re = q + dl;
          int64_t size = 0;
          while (r < re) {
            uint64_t t3;
            get_varint(r, re, &t3);
            if ((t3 >> 3) == 1 && (t3 & 7) == 0) { uint64_t sz; get_varint(r, re, &sz); size = (int64_t)sz; }
            else skip_field(r, re, (int)(t3 & 7));
          }
          e.shape.push_back(size);
          q = re;
        } else {
          skip_field(q, qe, (int)(t2 & 7));
        }
      }
      p = qe;
    } else if (f == 3 && wt == 0) { get_varint(p, end, &v); e.shard_id = (int)v; }
    else if (f == 4 && wt == 0) { get_varint(p, end, &v); e.offset = (int64_t)v; }
    else if (f == 5 && wt == 0) { get_varint(p, end, &v); e.size = (int64_t)v; }
    else if (f == 6 && wt == 5) { memcpy(&e.crc32c, p, 4); p += 4; }
    else skip_field(p, end, wt);
  }
  return e;
}

// ---- SSTable block builder ------------------------------------------------------------------
class BlockBuilder {
 public:
  explicit BlockBuilder(int restart_interval = 16) : interval_(restart_interval) { restarts_.push_back(0); }
  void add(const std::string& key, const std::string& value) {
    size_t shared = 0;
    if (counter_ < interval_) {
      const size_t mn = std::min(last_key_.size(), key.size());
      while (shared < mn && last_key_[shared] == key[shared]) ++shared;
    } else {
      restarts_.push_back((uint32_t)buf_.size());
      counter_ = 0;
    }
    put_varint(&buf_, shared);
    put_varint(&buf_, key.size() - shared);
    put_varint(&buf_, value.size());
    buf_.append(key.data() + shared, key.size() - shared);
    buf_.append(value);
    last_key_ = key;
    counter_++;
  }
  std::string finish() {
    for (uint32_t r : restarts_) put_fixed32(&buf_, r);
    put_fixed32(&buf_, (uint32_t)restarts_.size());
    return buf_;
  }
  size_t size() const { return buf_.size(); }
  bool empty() const { return buf_.empty(); }

 private:
  std::string buf_;
  std::vector<uint32_t> restarts_;
  int counter_ = 0;
  int interval_;
  std::string last_key_;
};

static std::string block_handle(uint64_t off, uint64_t size) {
  std::string s;
  put_varint(&s, off);
  put_varint(&s, size);
  return s;
}

// writes block + 5-byte trailer, returns handle
static std::string emit_block(std::string* file, const std::string& contents) {
  const uint64_t off = file->size();
  file->append(contents);
  const char type = 0;  // no compression
  uint32_t crc = crc32c(contents.data(), contents.size());
  crc = crc32c_extend(crc, &type, 1);
  file->push_back(type);
  put_fixed32(file, crc_mask(crc));
  return block_handle(off, contents.size());
}

static const uint64_t kTableMagic = 0xdb4775248b80fb57ull;

void write_bundle(const std::string& prefix, const std::vector<NamedTensor>& tensors) {
  // data file: tensors in key order (TF writes in Add() order, sorted keys required by the table)
  std::vector<const NamedTensor*> order;
  for (auto& t : tensors) order.push_back(&t);
  std::sort(order.begin(), order.end(), [](const NamedTensor* a, const NamedTensor* b) { return a->name < b->name; });
  for (size_t i = 1; i < order.size(); ++i)
    if (order[i]->name == order[i - 1]->name) throw std::runtime_error("bundle: duplicate key " + order[i]->name);
  std::string data;
  std::vector<std::pair<std::string, std::string>> kvs;
  kvs.emplace_back("", encode_header());
  for (const NamedTensor* t : order) {
    Entry e;
    e.dtype = t->dtype;
    e.shape = t->shape;
    e.offset = (int64_t)data.size();
    e.size = (int64_t)t->bytes.size();
    e.crc32c = crc_mask(crc32c(t->bytes.data(), t->bytes.size()));
    data.append(t->bytes);
    kvs.emplace_back(t->name, encode_entry(e));
  }
  // index (sstable)
  std::string file;
  BlockBuilder index_block(1);
  BlockBuilder cur;
  std::string last_key;
  for (auto& kv : kvs) {
    cur.add(kv.first, kv.second);
    last_key = kv.first;
    if (cur.size() >= (64u << 10)) {
      const std::string h = emit_block(&file, cur.finish());
      index_block.add(last_key, h);
      cur = BlockBuilder();
    }
  }
  if (!cur.empty()) {
    const std::string h = emit_block(&file, cur.finish());
    index_block.add(last_key, h);
  }
  BlockBuilder meta;
  const std::string meta_h = emit_block(&file, meta.finish());
  const std::string index_h = emit_block(&file, index_block.finish());
  std::string footer = meta_h + index_h;
  footer.resize(40, '\0');
  put_fixed64(&footer, kTableMagic);
  file.append(footer);

  const std::string dpath = prefix + ".data-00000-of-00001";
  const std::string ipath = prefix + ".index";
  {
    std::ofstream f(dpath + ".tmp", std::ios::binary);
    f.write(data.data(), (std::streamsize)data.size());
    if (!f) throw std::runtime_error("bundle: cannot write " + dpath);
  }
  {
    std::ofstream f(ipath + ".tmp", std::ios::binary);
    f.write(file.data(), (std::streamsize)file.size());
    if (!f) throw std::runtime_error("bundle: cannot write " + ipath);
  }
  if (rename((dpath + ".tmp").c_str(), dpath.c_str()) != 0 || rename((ipath + ".tmp").c_str(), ipath.c_str()) != 0)
    throw std::runtime_error("bundle: rename failed");
}

static std::string read_file(const std::string& path) {
  std::ifstream f(path, std::ios::binary);
  if (!f) throw std::runtime_error("bundle: cannot open " + path);
  return std::string((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
}

static void parse_block(const std::string& file, uint64_t off, uint64_t size,
                        std::vector<std::pair<std::string, std::string>>* out, bool verify) {
  if (off + size + 5 > file.size()) throw std::runtime_error("bundle: block out of range");
  const char* b = file.data() + off;
  if (verify) {
    uint32_t crc = crc32c(b, size);
    crc = crc32c_extend(crc, b + size, 1);
    uint32_t stored;
    memcpy(&stored, b + size + 1, 4);
    if (crc_unmask(stored) != crc) throw std::runtime_error("bundle: block checksum mismatch");
  }
  uint32_t nrest;
  memcpy(&nrest, b + size - 4, 4);
  const uint64_t limit = size - 4 - 4ull * nrest;
  const uint8_t* p = (const uint8_t*)b;
  const uint8_t* end = p + limit;
  std::string key;
  while (p < end) {
    uint64_t shared, nonshared, vlen;
    if (!get_varint(p, end, &shared) || !get_varint(p, end, &nonshared) || !get_varint(p, end, &vlen))
      throw std::runtime_error("bundle: corrupt block");
    key.resize(shared);
    key.append((const char*)p, nonshared);
    p += nonshared;
    out->emplace_back(key, std::string((const char*)p, vlen));
    p += vlen;
  }
}

std::map<std::string, Entry> read_index(const std::string& prefix) {
  const std::string file = read_file(prefix + ".index");
  if (file.size() < 48) throw std::runtime_error("bundle: index too small");
  uint64_t magic;
  memcpy(&magic, file.data() + file.size() - 8, 8);
  if (magic != kTableMagic) throw std::runtime_error("bundle: bad table magic");
  const uint8_t* p = (const uint8_t*)file.data() + file.size() - 48;
  const uint8_t* end = p + 40;
  uint64_t mo, ms, io, is;
  get_varint(p, end, &mo);
  get_varint(p, end, &ms);
  get_varint(p, end, &io);
  get_varint(p, end, &is);
  std::vector<std::pair<std::string, std::string>> idx;
  parse_block(file, io, is, &idx, true);
  std::map<std::string, Entry> out;
  for (auto& kv : idx) {
    const uint8_t* q = (const uint8_t*)kv.second.data();
    const uint8_t* qe = q + kv.second.size();
    uint64_t bo, bs;
    get_varint(q, qe, &bo);
    get_varint(q, qe, &bs);
    std::vector<std::pair<std::string, std::string>> entries;
    parse_block(file, bo, bs, &entries, true);
    for (auto& e : entries)
      if (!e.first.empty()) out[e.first] = decode_entry(e.second);
  }
  return out;
}

std::vector<NamedTensor> read_bundle(const std::string& prefix, bool verify_crc) {
  auto idx = read_index(prefix);
  const std::string data = read_file(prefix + ".data-00000-of-00001");
  std::vector<NamedTensor> out;
  for (auto& kv : idx) {
    const Entry& e = kv.second;
    if (e.offset + e.size > (int64_t)data.size()) throw std::runtime_error("bundle: entry out of range " + kv.first);
    NamedTensor t;
    t.name = kv.first;
    t.dtype = e.dtype;
    t.shape = e.shape;
    t.bytes.assign(data.data() + e.offset, (size_t)e.size);
    if (verify_crc && crc_unmask(e.crc32c) != crc32c(t.bytes.data(), t.bytes.size()))
      throw std::runtime_error("bundle: tensor checksum mismatch for " + kv.first);
    out.push_back(std::move(t));
  }
  return out;
}

}  // namespace ckpt
}  // namespace dtg
