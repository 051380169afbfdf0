// Native HDF5 (subset) reader/writer -- see h5.h for scope.
#include "h5.h"

#include <algorithm>
#include <cstring>
#include <fstream>
#include <functional>
#include <sstream>

namespace sml {
namespace h5 {
namespace {

constexpr uint64_t UNDEF = ~0ull;
const char kSig[8] = {'\x89', 'H', 'D', 'F', '\r', '\n', '\x1a', '\n'};

// ---------------------------------------------------------------------------
// bounds-checked little-endian reader
// ---------------------------------------------------------------------------
struct Buf {
  const uint8_t* p = nullptr;
  uint64_t n = 0;
  void need(uint64_t off, uint64_t len) const {
    if (off > n || len > n - off) throw Error("h5: truncated or corrupt file (read past end)");
  }
  uint64_t u(uint64_t off, int bytes) const {
    need(off, (uint64_t)bytes);
    uint64_t v = 0;
    for (int i = bytes - 1; i >= 0; --i) v = (v << 8) | p[off + i];
    return v;
  }
  std::string str(uint64_t off, uint64_t len) const {
    need(off, len);
    return std::string(reinterpret_cast<const char*>(p) + off, (size_t)len);
  }
  std::string cstr(uint64_t off, uint64_t limit) const {
    need(off, 1);
    uint64_t end = off;
    const uint64_t stop = std::min(n, limit);
    while (end < stop && p[end]) ++end;
    if (end >= stop) throw Error("h5: unterminated string in heap");
    return std::string(reinterpret_cast<const char*>(p) + off, (size_t)(end - off));
  }
  bool sig(uint64_t off, const char* s) const {
    if (off > n || n - off < 4) return false;
    return std::memcmp(p + off, s, 4) == 0;
  }
};

struct DType {
  int cls = -1;
  uint32_t size = 0;
  bool sign = false;
  bool big = false;
  int str_pad = 0, cset = 0;
  bool vlen_string = false;
};

struct Msg {
  int type;
  int flags;
  uint64_t off;
  uint64_t size;
};

class Reader {
 public:
  explicit Reader(const std::string& bytes) {
    b_.p = reinterpret_cast<const uint8_t*>(bytes.data());
    b_.n = bytes.size();
  }

  Node read() {
    uint64_t sb = UNDEF;
    for (uint64_t off = 0; off < b_.n && off <= (1ull << 30); off = off ? off * 2 : 512) {
      if (b_.n - off >= 8 && std::memcmp(b_.p + off, kSig, 8) == 0) { sb = off; break; }
    }
    if (sb == UNDEF) throw Error("h5: not an HDF5 file (signature not found)");
    const int ver = (int)b_.u(sb + 8, 1);
    if (ver > 1) throw Error("h5: superblock version " + std::to_string(ver) + " not supported (need 0/1)");
    so_ = (int)b_.u(sb + 13, 1);
    sl_ = (int)b_.u(sb + 14, 1);
    if ((so_ != 8 && so_ != 4) || (sl_ != 8 && sl_ != 4)) throw Error("h5: unsupported offset/length size");
    uint64_t p = sb + 16 + 4 + 4;   // after K values and consistency flags
    if (ver == 1) p += 4;            // indexed storage K + reserved
    base_ = b_.u(p, so_);
    p += 4 * so_;                    // base, free-space, EOF, driver info
    // root group symbol table entry
    const uint64_t root_oh = b_.u(p + so_, so_);
    return read_object(root_oh, 0);
  }

 private:
  Buf b_;
  int so_ = 8, sl_ = 8;
  uint64_t base_ = 0;
  std::map<uint64_t, std::map<uint32_t, std::pair<uint64_t, uint64_t>>> gheap_;

  uint64_t addr(uint64_t a) const { return a == UNDEF ? UNDEF : base_ + a; }

  std::vector<Msg> messages(uint64_t oh) {
    oh = addr(oh);
    std::vector<Msg> out;
    if (b_.sig(oh, "OHDR")) throw Error("h5: version-2 object headers not supported");
    const int ver = (int)b_.u(oh, 1);
    if (ver != 1) throw Error("h5: unknown object header version " + std::to_string(ver));
    const uint64_t nmsgs = b_.u(oh + 2, 2);
    const uint64_t hsize = b_.u(oh + 8, 4);
    std::vector<std::pair<uint64_t, uint64_t>> chunks{{oh + 16, hsize}};
    uint64_t count = 0;
    for (size_t ci = 0; ci < chunks.size() && count < nmsgs; ++ci) {
      if (ci > 64) throw Error("h5: too many continuation blocks");
      uint64_t pos = chunks[ci].first;
      const uint64_t end = chunks[ci].first + chunks[ci].second;
      b_.need(chunks[ci].first, chunks[ci].second);
      while (pos + 8 <= end && count < nmsgs) {
        const int type = (int)b_.u(pos, 2);
        const uint64_t size = b_.u(pos + 2, 2);
        const int flags = (int)b_.u(pos + 4, 1);
        const uint64_t data = pos + 8;
        if (data + size > end) throw Error("h5: object header message overruns its block");
        if (type == 0x10) {
          chunks.emplace_back(addr(b_.u(data, so_)), b_.u(data + so_, sl_));
        } else {
          out.push_back(Msg{type, flags, data, size});
        }
        ++count;
        pos = data + size;
      }
    }
    return out;
  }

  DType datatype(uint64_t off, uint64_t* consumed = nullptr) {
    DType t;
    const int b0 = (int)b_.u(off, 1);
    t.cls = b0 & 0x0f;
    const uint64_t bf = b_.u(off + 1, 3);
    t.size = (uint32_t)b_.u(off + 4, 4);
    uint64_t used = 8;
    switch (t.cls) {
      case 0:  // fixed-point
        t.big = bf & 1;
        t.sign = (bf >> 3) & 1;
        used += 4;
        break;
      case 1:  // floating point
        t.big = bf & 1;
        used += 12;
        if (t.size != 4 && t.size != 8 && t.size != 2) throw Error("h5: unsupported float size");
        break;
      case 3:  // fixed string
        t.str_pad = (int)(bf & 0x0f);
        t.cset = (int)((bf >> 4) & 0x0f);
        break;
      case 9: {  // variable length
        const int vt = (int)(bf & 0x0f);
        t.str_pad = (int)((bf >> 4) & 0x0f);
        t.cset = (int)((bf >> 8) & 0x0f);
        uint64_t base_used = 0;
        datatype(off + 8, &base_used);
        used += base_used;
        if (vt != 1) throw Error("h5: variable-length sequences are not supported (only strings)");
        t.vlen_string = true;
        break;
      }
      default:
        throw Error("h5: unsupported datatype class " + std::to_string(t.cls));
    }
    if (consumed) *consumed = used;
    return t;
  }

  void dataspace(uint64_t off, Value& v) {
    const int ver = (int)b_.u(off, 1);
    const int rank = (int)b_.u(off + 1, 1);
    const int flags = (int)b_.u(off + 2, 1);
    uint64_t p;
    v.shape.clear();
    v.is_null = false;
    if (ver == 1) {
      p = off + 8;
    } else if (ver == 2) {
      const int type = (int)b_.u(off + 3, 1);
      if (type == 2) v.is_null = true;
      p = off + 4;
    } else {
      throw Error("h5: unknown dataspace version");
    }
    (void)flags;
    for (int i = 0; i < rank; ++i) v.shape.push_back(b_.u(p + (uint64_t)i * sl_, sl_));
  }

  std::string gheap_object(uint64_t coll, uint32_t index) {
    coll = addr(coll);
    auto it = gheap_.find(coll);
    if (it == gheap_.end()) {
      if (!b_.sig(coll, "GCOL")) throw Error("h5: bad global heap collection");
      const uint64_t csize = b_.u(coll + 8, sl_);
      b_.need(coll, csize);
      std::map<uint32_t, std::pair<uint64_t, uint64_t>> objs;
      uint64_t p = coll + 8 + sl_;
      const uint64_t end = coll + csize;
      while (p + 8 + sl_ <= end) {
        const uint32_t idx = (uint32_t)b_.u(p, 2);
        const uint64_t osize = b_.u(p + 8, sl_);
        if (idx == 0) break;  // free space
        const uint64_t data = p + 8 + sl_;
        if (data + osize > end) throw Error("h5: global heap object overruns collection");
        objs[idx] = {data, osize};
        p = data + ((osize + 7) & ~7ull);
      }
      it = gheap_.emplace(coll, std::move(objs)).first;
    }
    auto jt = it->second.find(index);
    if (jt == it->second.end()) throw Error("h5: global heap object not found");
    return b_.str(jt->second.first, jt->second.second);
  }

  void decode(const DType& t, uint64_t data, Value& v) {
    const uint64_t n = v.count();
    if (t.vlen_string) {
      v.kind = Value::VLEN_STRING;
      v.cset = t.cset;
      const uint64_t es = 4 + so_ + 4;
      v.strings.clear();
      for (uint64_t i = 0; i < n; ++i) {
        const uint64_t e = data + i * es;
        const uint64_t len = b_.u(e, 4);
        const uint64_t coll = b_.u(e + 4, so_);
        const uint32_t idx = (uint32_t)b_.u(e + 4 + so_, 4);
        if (coll == 0 && len == 0) { v.strings.emplace_back(); continue; }
        std::string s = gheap_object(coll, idx);
        if (len < s.size()) s.resize((size_t)len);
        v.strings.push_back(std::move(s));
      }
      return;
    }
    const uint64_t bytes = n * t.size;
    std::string raw = b_.str(data, bytes);
    if (t.cls == 3) {
      v.kind = Value::FIXED_STRING;
      v.itemsize = (int)t.size;
      v.str_pad = t.str_pad;
      v.cset = t.cset;
      v.data = std::move(raw);
      return;
    }
    v.kind = Value::NUMERIC;
    v.itemsize = (int)t.size;
    v.dtype = t.cls == 1 ? 'f' : (t.sign ? 'i' : 'u');
    if (t.big && t.size > 1) {
      for (uint64_t i = 0; i < n; ++i) std::reverse(raw.begin() + i * t.size, raw.begin() + (i + 1) * t.size);
    }
    v.data = std::move(raw);
  }

  std::pair<std::string, Value> attribute(const Msg& m) {
    const uint64_t o = m.off;
    const int ver = (int)b_.u(o, 1);
    const uint64_t name_size = b_.u(o + 2, 2);
    const uint64_t dt_size = b_.u(o + 4, 2);
    const uint64_t ds_size = b_.u(o + 6, 2);
    uint64_t p;
    auto pad8 = [](uint64_t x) { return (x + 7) & ~7ull; };
    std::string name;
    uint64_t dt_off, ds_off, data;
    if (ver == 1) {
      p = o + 8;
      name = b_.cstr(p, p + name_size);
      dt_off = p + pad8(name_size);
      ds_off = dt_off + pad8(dt_size);
      data = ds_off + pad8(ds_size);
    } else if (ver == 2 || ver == 3) {
      p = o + 8 + (ver == 3 ? 1 : 0);
      name = b_.cstr(p, p + name_size);
      dt_off = p + name_size;
      ds_off = dt_off + dt_size;
      data = ds_off + ds_size;
    } else {
      throw Error("h5: unknown attribute message version");
    }
    if ((int)b_.u(o + 1, 1) & 0x3 && ver >= 2) throw Error("h5: shared attribute datatypes not supported");
    Value v;
    const DType t = datatype(dt_off);
    dataspace(ds_off, v);
    decode(t, data, v);
    return {name, std::move(v)};
  }

  void walk_btree(uint64_t bt, uint64_t heap_data, uint64_t heap_end,
                  std::vector<std::pair<std::string, uint64_t>>& out, int depth) {
    if (depth > 32) throw Error("h5: B-tree too deep");
    bt = addr(bt);
    if (!b_.sig(bt, "TREE")) throw Error("h5: bad group B-tree node");
    if (b_.u(bt + 4, 1) != 0) throw Error("h5: B-tree is not a group node");
    const int level = (int)b_.u(bt + 5, 1);
    const uint64_t used = b_.u(bt + 6, 2);
    const uint64_t kc = bt + 8 + 2 * so_;
    for (uint64_t i = 0; i < used; ++i) {
      const uint64_t child = b_.u(kc + sl_ + i * (sl_ + so_), so_);
      if (level > 0) {
        walk_btree(child, heap_data, heap_end, out, depth + 1);
      } else {
        const uint64_t sn = addr(child);
        if (!b_.sig(sn, "SNOD")) throw Error("h5: bad symbol table node");
        const uint64_t nsyms = b_.u(sn + 6, 2);
        const uint64_t esz = 2 * so_ + 24;
        for (uint64_t k = 0; k < nsyms; ++k) {
          const uint64_t e = sn + 8 + k * esz;
          const uint64_t name_off = b_.u(e, so_);
          const uint64_t oh = b_.u(e + so_, so_);
          out.emplace_back(b_.cstr(heap_data + name_off, heap_end), oh);
        }
      }
    }
  }

  Node read_object(uint64_t oh, int depth) {
    if (depth > 64) throw Error("h5: group nesting too deep (cycle?)");
    const std::vector<Msg> msgs = messages(oh);
    Node node;
    const Msg* symtab = nullptr;
    const Msg* layout = nullptr;
    const Msg* dtype = nullptr;
    const Msg* dspace = nullptr;
    for (const Msg& m : msgs) {
      switch (m.type) {
        case 0x11: symtab = &m; break;
        case 0x08: layout = &m; break;
        case 0x03: dtype = &m; break;
        case 0x01: dspace = &m; break;
        case 0x0C: node.attrs.push_back(attribute(m)); break;
        case 0x06: throw Error("h5: link messages (new-style groups) not supported");
        default: break;
      }
      if ((m.type == 0x03 || m.type == 0x01) && (m.flags & 0x02)) throw Error("h5: shared messages not supported");
    }
    if (symtab) {
      node.is_group = true;
      const uint64_t bt = b_.u(symtab->off, so_);
      const uint64_t heap = addr(b_.u(symtab->off + so_, so_));
      if (!b_.sig(heap, "HEAP")) throw Error("h5: bad local heap");
      const uint64_t dsize = b_.u(heap + 8, sl_);
      const uint64_t daddr = addr(b_.u(heap + 8 + 2 * sl_, so_));
      b_.need(daddr, dsize);
      std::vector<std::pair<std::string, uint64_t>> entries;
      walk_btree(bt, daddr, daddr + dsize, entries, 0);
      for (auto& e : entries) node.children.emplace_back(e.first, read_object(e.second, depth + 1));
      return node;
    }
    if (!layout || !dtype || !dspace) throw Error("h5: object is neither group nor dataset");
    node.is_group = false;
    Value& v = node.value;
    dataspace(dspace->off, v);
    const DType t = datatype(dtype->off);
    const uint64_t lo = layout->off;
    const int lver = (int)b_.u(lo, 1);
    uint64_t data = UNDEF;
    std::string compact;
    if (lver == 3) {
      const int cls = (int)b_.u(lo + 1, 1);
      if (cls == 0) {
        const uint64_t sz = b_.u(lo + 2, 2);
        data = lo + 4;
        b_.need(data, sz);
      } else if (cls == 1) {
        data = addr(b_.u(lo + 2, so_));
      } else {
        throw Error("h5: chunked datasets not supported");
      }
    } else if (lver == 1 || lver == 2) {
      const int cls = (int)b_.u(lo + 2, 1);
      if (cls == 1) data = addr(b_.u(lo + 8, so_));
      else throw Error("h5: only contiguous v1/v2 layouts supported");
    } else {
      throw Error("h5: unknown layout version");
    }
    if (data == UNDEF) {
      // never written: libhdf5 semantics = fill value (zeros)
      std::string zeros(v.count() * (t.vlen_string ? (8 + so_) : t.size), '\0');
      Value tmp = v;
      if (t.vlen_string) { tmp.kind = Value::VLEN_STRING; tmp.strings.assign(v.count(), std::string()); v = tmp; }
      else { v.kind = t.cls == 3 ? Value::FIXED_STRING : Value::NUMERIC; v.itemsize = (int)t.size;
             v.dtype = t.cls == 1 ? 'f' : (t.sign ? 'i' : 'u'); v.data = zeros; }
      return node;
    }
    decode(t, data, v);
    return node;
  }
};

// ---------------------------------------------------------------------------
// writer
// ---------------------------------------------------------------------------
class Writer {
 public:
  std::string run(const Node& root) {
    if (!root.is_group) throw Error("h5: root must be a group");
    out_.assign(96, '\0');  // superblock v0 with 8-byte offsets/lengths
    collect_strings(root);
    write_global_heap();
    GroupInfo gi;
    const uint64_t root_oh = write_group(root, &gi);
    // superblock
    std::memcpy(&out_[0], kSig, 8);
    out_[8] = 0;   // superblock version
    out_[9] = 0;   // free-space version
    out_[10] = 0;  // root group symbol table entry version
    out_[11] = 0;
    out_[12] = 0;  // shared header message format version
    out_[13] = 8;  // sizeof offsets
    out_[14] = 8;  // sizeof lengths
    out_[15] = 0;
    put(16, 4, 2);   // group leaf node K
    put(18, 16, 2);  // group internal node K
    put(20, 0, 4);   // consistency flags
    put(24, 0, 8);   // base address
    put(32, UNDEF, 8);
    put(40, out_.size(), 8);  // end of file address
    put(48, UNDEF, 8);        // driver info
    // root symbol table entry
    put(56, 0, 8);            // link name offset
    put(64, root_oh, 8);
    put(72, 1, 4);            // cache type 1: scratch holds B-tree + heap
    put(76, 0, 4);
    put(80, gi.btree, 8);
    put(88, gi.heap, 8);
    return out_;
  }

 private:
  std::string out_;
  std::vector<std::string> vstrings_;

  struct GroupInfo {
    uint64_t btree = UNDEF, heap = UNDEF;
  };

  void put(uint64_t off, uint64_t v, int bytes) {
    for (int i = 0; i < bytes; ++i) out_[off + i] = (char)((v >> (8 * i)) & 0xff);
  }
  uint64_t alloc(uint64_t n) {
    uint64_t a = (out_.size() + 7) & ~7ull;
    out_.resize(a + n, '\0');
    return a;
  }
  static void app(std::string& s, uint64_t v, int bytes) {
    for (int i = 0; i < bytes; ++i) s.push_back((char)((v >> (8 * i)) & 0xff));
  }
  static void pad8(std::string& s) {
    while (s.size() % 8) s.push_back('\0');
  }

  void collect_value(const Value& v) {
    if (v.kind == Value::VLEN_STRING)
      for (const auto& s : v.strings) vstrings_.push_back(s);
  }
  void collect_strings(const Node& n) {
    for (const auto& a : n.attrs) collect_value(a.second);
    if (n.is_group) {
      for (const auto& c : n.children) collect_strings(c.second);
    } else {
      collect_value(n.value);
    }
  }

  // one global heap collection (>= 4096 bytes) holding every vlen string
  uint64_t gcol_ = UNDEF;
  std::map<std::string, uint32_t> gidx_;  // string content -> heap object index
  void write_global_heap() {
    if (vstrings_.empty()) return;
    std::string body;
    uint32_t idx = 1;
    for (const auto& s : vstrings_) {
      if (gidx_.count(s)) continue;  // identical strings share one heap object
      app(body, idx, 2);
      app(body, 1, 2);   // reference count
      app(body, 0, 4);
      app(body, s.size(), 8);
      body += s;
      pad8(body);
      gidx_[s] = idx++;
    }
    uint64_t total = 16 + body.size();
    uint64_t csize = std::max<uint64_t>(4096, ((total + 16 + 4095) / 4096) * 4096);
    std::string coll = "GCOL";
    app(coll, 1, 1);
    app(coll, 0, 3);
    app(coll, csize, 8);
    coll += body;
    const uint64_t free_sz = csize - coll.size();
    app(coll, 0, 2);  // free-space object (index 0)
    app(coll, 0, 2);
    app(coll, 0, 4);
    app(coll, free_sz, 8);
    coll.resize(csize, '\0');
    gcol_ = alloc(csize);
    std::memcpy(&out_[gcol_], coll.data(), coll.size());
  }

  // ---- datatypes ----------------------------------------------------------
  static std::string dt_numeric(char kind, int size) {
    std::string d;
    if (kind == 'f') {
      d.push_back(0x11);
      d.push_back(0x20);
      d.push_back((char)(size * 8 - 1));
      d.push_back(0);
      app(d, size, 4);
      app(d, 0, 2);
      app(d, size * 8, 2);
      if (size == 4) { d.push_back(23); d.push_back(8); d.push_back(0); d.push_back(23); app(d, 127, 4); }
      else if (size == 8) { d.push_back(52); d.push_back(11); d.push_back(0); d.push_back(52); app(d, 1023, 4); }
      else if (size == 2) { d.push_back(10); d.push_back(5); d.push_back(0); d.push_back(10); app(d, 15, 4); }
      else throw Error("h5: unsupported float size for writing");
    } else {
      d.push_back(0x10);
      d.push_back(kind == 'i' ? 0x08 : 0x00);
      d.push_back(0);
      d.push_back(0);
      app(d, size, 4);
      app(d, 0, 2);
      app(d, size * 8, 2);
    }
    return d;
  }
  static std::string dt_fixed_string(int size, int pad, int cset) {
    std::string d;
    d.push_back(0x13);
    d.push_back((char)((pad & 0xf) | ((cset & 0xf) << 4)));
    d.push_back(0);
    d.push_back(0);
    app(d, size, 4);
    return d;
  }
  static std::string dt_vlen_string(int cset) {
    std::string d;
    d.push_back(0x19);
    d.push_back(0x01);          // type = string, padding = null-terminate
    d.push_back((char)(cset & 0xf));
    d.push_back(0);
    app(d, 16, 4);              // 4-byte length + 8-byte collection address + 4-byte index
    // base type: 1-byte unsigned fixed-point -- byte-identical to what h5py 2.x
    // wrote for the reference models/*.h5 string attributes
    d += dt_numeric('u', 1);
    return d;
  }
  static std::string dtype_of(const Value& v) {
    switch (v.kind) {
      case Value::NUMERIC: return dt_numeric(v.dtype, v.itemsize);
      case Value::FIXED_STRING: return dt_fixed_string(v.itemsize, v.str_pad, v.cset);
      case Value::VLEN_STRING: return dt_vlen_string(v.cset);
    }
    throw Error("h5: bad value kind");
  }
  static std::string dataspace_of(const Value& v) {
    std::string d;
    d.push_back(1);  // version 1
    d.push_back((char)v.shape.size());
    d.push_back(0);  // flags: no max dims
    d.push_back(0);
    app(d, 0, 4);
    for (auto x : v.shape) app(d, x, 8);
    return d;
  }
  std::string payload_of(const Value& v) {
    if (v.kind != Value::VLEN_STRING) {
      const uint64_t need = v.count() * (uint64_t)v.itemsize;
      if (v.data.size() != need) throw Error("h5: value byte size does not match its shape");
      return v.data;
    }
    if (v.strings.size() != v.count()) throw Error("h5: vlen string count does not match shape");
    std::string d;
    for (const auto& s : v.strings) {
      app(d, s.size(), 4);
      app(d, gcol_, 8);
      app(d, gidx_.at(s), 4);
    }
    return d;
  }

  // ---- object headers -----------------------------------------------------
  static void add_msg(std::string& msgs, int type, int flags, const std::string& data) {
    std::string d = data;
    pad8(d);
    if (d.size() > 0xffff) throw Error("h5: header message too large");
    app(msgs, type, 2);
    app(msgs, d.size(), 2);
    msgs.push_back((char)flags);
    msgs.append(3, '\0');
    msgs += d;
  }
  std::string attr_msg(const std::string& name, const Value& v) {
    std::string dt = dtype_of(v), ds = dataspace_of(v), pl = payload_of(v);
    std::string m;
    m.push_back(1);
    m.push_back(0);
    app(m, name.size() + 1, 2);
    app(m, dt.size(), 2);
    app(m, ds.size(), 2);
    std::string nm = name;
    nm.push_back('\0');
    pad8(nm);
    m += nm;
    pad8(dt);
    m += dt;
    pad8(ds);
    m += ds;
    m += pl;
    return m;
  }
  uint64_t write_header(int nmsgs, const std::string& msgs) {
    const uint64_t a = alloc(16 + msgs.size());
    put(a, 1, 1);
    put(a + 1, 0, 1);
    put(a + 2, (uint64_t)nmsgs, 2);
    put(a + 4, 1, 4);   // reference count
    put(a + 8, msgs.size(), 4);
    std::memcpy(&out_[a + 16], msgs.data(), msgs.size());
    return a;
  }

  uint64_t write_dataset(const Node& n) {
    const Value& v = n.value;
    const std::string pl = payload_of(v);
    const uint64_t data = pl.empty() ? UNDEF : alloc(pl.size());
    if (!pl.empty()) std::memcpy(&out_[data], pl.data(), pl.size());
    std::string msgs;
    int cnt = 0;
    add_msg(msgs, 0x01, 0, dataspace_of(v)); ++cnt;
    add_msg(msgs, 0x03, 1, dtype_of(v)); ++cnt;
    std::string fill;
    fill.push_back(2);  // fill value message v2
    fill.push_back(2);  // space allocation time: late
    fill.push_back(2);  // fill write time: if set
    fill.push_back(0);  // fill value undefined
    add_msg(msgs, 0x05, 1, fill); ++cnt;
    std::string lay;
    lay.push_back(3);   // layout v3
    lay.push_back(1);   // contiguous
    app(lay, data, 8);
    app(lay, pl.size(), 8);
    add_msg(msgs, 0x08, 0, lay); ++cnt;
    for (const auto& a : n.attrs) { add_msg(msgs, 0x0C, 0, attr_msg(a.first, a.second)); ++cnt; }
    return write_header(cnt, msgs);
  }

  uint64_t write_group(const Node& n, GroupInfo* gi) {
    // children first (post-order), sorted by name as the symbol table requires
    struct Child {
      std::string name;
      uint64_t oh;
      bool group;
      GroupInfo info;
    };
    std::vector<Child> kids;
    for (const auto& c : n.children) {
      Child k{c.first, 0, c.second.is_group, {}};
      if (c.first.empty() || c.first.find('/') != std::string::npos) throw Error("h5: bad link name '" + c.first + "'");
      k.oh = c.second.is_group ? write_group(c.second, &k.info) : write_dataset(c.second);
      kids.push_back(std::move(k));
    }
    std::sort(kids.begin(), kids.end(), [](const Child& x, const Child& y) { return x.name < y.name; });
    for (size_t i = 1; i < kids.size(); ++i)
      if (kids[i].name == kids[i - 1].name) throw Error("h5: duplicate link name " + kids[i].name);
    if (kids.size() > 8 * 32) throw Error("h5: more than 256 links in one group not supported");
    // local heap data segment: "" at 0, then names
    std::string heap;
    heap.append(8, '\0');
    std::vector<uint64_t> name_off;
    for (const auto& k : kids) {
      name_off.push_back(heap.size());
      heap += k.name;
      heap.push_back('\0');
      pad8(heap);
    }
    const uint64_t heap_data = alloc(heap.size());
    std::memcpy(&out_[heap_data], heap.data(), heap.size());
    const uint64_t hh = alloc(32);
    std::memcpy(&out_[hh], "HEAP", 4);
    put(hh + 4, 0, 1);
    put(hh + 8, heap.size(), 8);
    put(hh + 16, UNDEF, 8);  // no free block
    put(hh + 24, heap_data, 8);
    // symbol table nodes (2K = 8 entries each)
    const uint64_t nsnod = kids.empty() ? 0 : (kids.size() + 7) / 8;
    std::vector<uint64_t> snods;
    for (uint64_t s = 0; s < nsnod; ++s) {
      const uint64_t a = alloc(8 + 8 * 40);
      std::memcpy(&out_[a], "SNOD", 4);
      put(a + 4, 1, 1);
      const uint64_t lo = s * 8, hi = std::min<uint64_t>(kids.size(), lo + 8);
      put(a + 6, hi - lo, 2);
      for (uint64_t i = lo; i < hi; ++i) {
        const uint64_t e = a + 8 + (i - lo) * 40;
        put(e, name_off[i], 8);
        put(e + 8, kids[i].oh, 8);
        if (kids[i].group) {
          put(e + 16, 1, 4);
          put(e + 24, kids[i].info.btree, 8);
          put(e + 32, kids[i].info.heap, 8);
        }
      }
      snods.push_back(a);
    }
    // one B-tree leaf node (K = 16 -> up to 32 children)
    const uint64_t bt = alloc(24 + 33 * 8 + 32 * 8);
    std::memcpy(&out_[bt], "TREE", 4);
    put(bt + 4, 0, 1);
    put(bt + 5, 0, 1);
    put(bt + 6, nsnod, 2);
    put(bt + 8, UNDEF, 8);
    put(bt + 16, UNDEF, 8);
    uint64_t p = bt + 24;
    put(p, 0, 8);  // key 0: empty string
    p += 8;
    for (uint64_t s = 0; s < nsnod; ++s) {
      put(p, snods[s], 8);
      p += 8;
      const uint64_t last = std::min<uint64_t>(kids.size(), (s + 1) * 8) - 1;
      put(p, name_off[last], 8);
      p += 8;
    }
    std::string msgs;
    int cnt = 0;
    std::string st;
    app(st, bt, 8);
    app(st, hh, 8);
    add_msg(msgs, 0x11, 0, st); ++cnt;
    for (const auto& a : n.attrs) { add_msg(msgs, 0x0C, 0, attr_msg(a.first, a.second)); ++cnt; }
    gi->btree = bt;
    gi->heap = hh;
    return write_header(cnt, msgs);
  }
};

}  // namespace

Node read_bytes(const std::string& bytes) { return Reader(bytes).read(); }

Node read_file(const std::string& path) {
  std::ifstream f(path, std::ios::binary);
  if (!f) throw Error("h5: cannot open " + path);
  std::stringstream ss;
  ss << f.rdbuf();
  return read_bytes(ss.str());
}

std::string write_bytes(const Node& root) { return Writer().run(root); }

void write_file(const std::string& path, const Node& root) {
  const std::string bytes = write_bytes(root);
  std::ofstream f(path, std::ios::binary | std::ios::trunc);
  if (!f) throw Error("h5: cannot create " + path);
  f.write(bytes.data(), (std::streamsize)bytes.size());
  if (!f) throw Error("h5: write failed for " + path);
}

}  // namespace h5
}  // namespace sml
