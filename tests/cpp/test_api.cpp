// test_api — the C++ surface (include/mtbl.hpp) exercised like the reference's own tests:
//   src/writer.rs:272-305 (empty, one_key, bytes_shortest_separator), examples/dump.rs and
//   get-key.rs behaviour, ReaderIntoIter's Get/Prefix/Range/From filters (src/reader.rs:385-402),
//   snappy files (src/compression.rs), and the error / panic mapping (src/error.rs, reader.rs:73).
// Runs on the GPU (blocks decode on the device).  Prints "OK <n>" on success, exits 1 on failure.
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "mtbl.hpp"

static int g_checks = 0;
#define CHECK(c)                                                        \
  do {                                                                  \
    ++g_checks;                                                         \
    if (!(c)) {                                                         \
      std::fprintf(stderr, "%s:%d: CHECK failed: %s\n", __FILE__, __LINE__, #c); \
      std::exit(1);                                                     \
    }                                                                   \
  } while (0)

using mtbl::Bytes;
static Bytes B(const std::string& s) { return Bytes(s.begin(), s.end()); }
static std::string S(const uint8_t* p, size_t n) { return std::string(reinterpret_cast<const char*>(p), n); }

// cfg1 records (examples/dump.rs plumbing): key "{:010}", value "{:010}" x (1 + i % 8)
static std::vector<std::pair<std::string, std::string>> cfg1(int n) {
  std::vector<std::pair<std::string, std::string>> v;
  char k[16];
  for (int i = 0; i < n; ++i) {
    std::snprintf(k, sizeof k, "%010d", i);
    std::string val;
    for (int r = 0; r < 1 + i % 8; ++r) val += k;
    v.emplace_back(k, val);
  }
  return v;
}

static Bytes write_file(const std::vector<std::pair<std::string, std::string>>& recs, mtbl::CompressionType c,
                        uint64_t block_size) {
  mtbl::Writer w = mtbl::WriterBuilder().compression_type(c).block_size(block_size).memory();
  for (const auto& kv : recs) w.insert(kv.first, kv.second);
  return w.into_inner();
}

static void test_empty() {   // src/writer.rs:276-284
  const Bytes vec = mtbl::Writer::memory().into_inner();
  const mtbl::Reader reader = mtbl::Reader::open(vec);
  auto iter = reader.into_iter();
  CHECK(!iter.next().has_value());
  CHECK(reader.metadata().count_entries == 0);
}

static void test_one_key() {   // src/writer.rs:286-298
  mtbl::Writer w = mtbl::WriterBuilder().memory();
  w.insert("hello", "I'm the one");
  const Bytes vec = w.into_inner();
  const mtbl::Reader reader = mtbl::Reader::open(vec);
  int count = 0;
  auto iter = reader.into_iter();
  while (auto r = iter.next()) {
    CHECK(S(r->key, r->key_len) == "hello" && S(r->val, r->val_len) == "I'm the one");
    ++count;
  }
  CHECK(count == 1);
  CHECK(reader.get("hello").value() == B("I'm the one"));
  CHECK(!reader.get("hell").has_value() && !reader.get("hello!").has_value());
}

static void test_separator_short() {   // src/writer.rs:300-305: keys whose separator hits the short-limit case
  mtbl::Writer w = mtbl::WriterBuilder().block_size(1024).memory();
  const std::string big(1100, 'x');
  w.insert("1st", big);   // flushes before "2": separator(start="1st", limit="2")
  w.insert("2", "y");
  const mtbl::Reader r = mtbl::Reader::open(w.into_inner());
  CHECK(r.len() == 2 && r.metadata().count_data_blocks == 2);
  CHECK(r.get("1st").value().size() == 1100 && r.get("2").value() == B("y"));
}

static void test_out_of_order() {   // src/writer.rs:118-123: "out-of-order key" panic
  mtbl::Writer w = mtbl::Writer::memory();
  w.insert("b", "1");
  bool panicked = false;
  try { w.insert("a", "2"); } catch (const mtbl::Panic&) { panicked = true; }
  CHECK(panicked);
}

static void test_cfg1(mtbl::CompressionType c) {   // examples/dump.rs + get-key.rs over cfg1
  const auto recs = cfg1(10000);
  const Bytes file = write_file(recs, c, 4096);
  const mtbl::Reader reader = mtbl::Reader::open(file);
  const mtbl::Metadata m = reader.metadata();
  CHECK(m.count_entries == recs.size() && m.compression_algorithm == static_cast<uint64_t>(c));
  CHECK(m.count_data_blocks > 100);
  size_t i = 0;
  auto iter = reader.into_iter();
  while (auto r = iter.next()) {
    CHECK(i < recs.size());
    CHECK(S(r->key, r->key_len) == recs[i].first && S(r->val, r->val_len) == recs[i].second);
    ++i;
  }
  CHECK(i == recs.size());
  for (size_t q : {size_t(0), size_t(1), size_t(4095), size_t(9999)}) CHECK(reader.get(recs[q].first).value() == B(recs[q].second));
  CHECK(!reader.get("0000000000x").has_value() && !reader.get("x").has_value() && !reader.get("").has_value());
  // GetPrefix: "00000012" -> keys 1200..1299
  auto p = reader.iter_prefix(B("00000012")).collect();
  CHECK(p.size() == 100 && p[0].first == B("0000001200") && p[99].first == B("0000001299"));
  // GetRange (end inclusive)
  auto g = reader.iter_range(B("0000000500"), B("0000000600")).collect();
  CHECK(g.size() == 101 && Bytes(g.back().second.begin(), g.back().second.begin() + 10) == B("0000000600"));
  // From
  auto f = reader.iter_from(B("0000009990")).collect();
  CHECK(f.size() == 10 && f[0].first == B("0000009990"));
  CHECK(reader.iter_prefix(B("x")).collect().empty() && reader.iter_from(B("1")).collect().empty());
  // ReaderIntoIter::seek (src/reader.rs:302-335)
  auto it = reader.iter_from(B("0000005000"));
  auto r0 = it.next();
  CHECK(r0 && S(r0->key, r0->key_len) == "0000005000");
  // another block: loaded and seeked to the landed SEPARATOR (src/reader.rs:305,328); between
  // keys that differ only in their last digit it is the block's last key
  CHECK(it.seek(B("0000009000")));
  auto r1 = it.next();
  CHECK(r1 && S(r1->key, r1->key_len) >= "0000009000");
  const std::string k1 = S(r1->key, r1->key_len);
  auto r2 = it.next();
  CHECK(r2 && std::stoll(S(r2->key, r2->key_len)) == std::stoll(k1) + 1);   // the next block's first
  // block_offset is now 9000's block: a seek into block 0 reloads block 0, seeked to its
  // separator (its last key)
  CHECK(it.seek(B("0000000003")));
  auto r3 = it.next();
  CHECK(r3 && S(r3->key, r3->key_len) > "0000000003" && S(r3->key, r3->key_len) < "0000000100");
  // the block_offset quirk: a fresh iter_from keeps block_offset 0, so seeking into block 0
  // (offset 0) re-seeks the block it holds instead of loading block 0
  auto q = reader.iter_from(B("0000005000"));
  (void)q.next();
  CHECK(q.seek(B("0000000003")));
  auto r4 = q.next();
  CHECK(r4 && S(r4->key, r4->key_len) != "0000000003" && S(r4->key, r4->key_len) <= "0000005000");
  CHECK(q.seek(B("zzz")) && !q.next().has_value());   // past the last key
}

// the hand-derived vectors of tests/golden/kat.json (seek_kat, make_golden.py): separators
// equal to the last key, bumped, and appended by write_u16 (src/writer.rs:239-265)
static void test_seek_kat() {
  const char* keys[] = {"key-0000", "key-0001", "key-0002", "key-0003", "key-0004", "key-0005",
                        "key-0007", "key-0008", "key-0009ab", "key-000:ac", "key-000;"};
  mtbl::Writer w = mtbl::WriterBuilder().block_size(1024).block_restart_interval(16).memory();
  for (int i = 0; i < 11; ++i) w.insert(std::string(keys[i]), std::string(300, (char)(0x41 + i)));
  const mtbl::Reader r = mtbl::Reader::open(w.into_inner());
  CHECK(r.metadata().count_data_blocks == 4);
  auto keys_of = [](mtbl::ReaderIntoIter& it, int n) {
    std::vector<std::string> out;
    for (int i = 0; i < n; ++i) {
      auto x = it.next();
      if (!x) break;
      out.push_back(S(x->key, x->key_len));
    }
    return out;
  };
  using V = std::vector<std::string>;
  {
    auto it = r.into_iter();
    it.seek(B("key-0001"));
    CHECK((keys_of(it, 3) == V{"key-0002", "key-0003", "key-0004"}));
  }
  {
    auto it = r.into_iter();
    it.seek(B("key-0004"));
    CHECK((keys_of(it, 2) == V{"key-0007", "key-0008"}));
  }
  {
    auto it = r.into_iter();
    it.seek(B("key-0008"));
    CHECK((keys_of(it, 1) == V{"key-000:ac"}));
  }
  {
    auto it = r.into_iter();
    it.seek(B("key-000;"));
    CHECK((keys_of(it, 2) == V{"key-000;"}));
    it.seek(B("key-000<"));
    CHECK(keys_of(it, 1).empty());
  }
  {
    auto it = r.iter_from(B("key-0005"));
    CHECK((keys_of(it, 3) == V{"key-0005", "key-0007", "key-0008"}));
    it.seek(B("key-0000"));
    CHECK((keys_of(it, 4) == V{"key-0007", "key-0008", "key-0009ab", "key-0003"}));
  }
}

static void test_errors() {
  const Bytes good = write_file(cfg1(2000), mtbl::CompressionType::None, 1024);
  // a file shorter than the footer: InvalidMetadataSize (src/reader.rs:35-37)
  bool err = false;
  try { (void)mtbl::Reader::open(Bytes(100, 0)); } catch (const mtbl::Error& e) { err = e.kind == mtbl::MtblError::InvalidMetadataSize; }
  CHECK(err);
  // a flipped byte inside the first data block: the checksum assert panics on iteration (src/reader.rs:159-164)
  Bytes bad = good;
  bad[40] ^= 0x5a;
  bool panicked = false;
  size_t yielded = 0;
  try {
    const mtbl::Reader r = mtbl::Reader::open(bad);
    auto it = r.into_iter();
    while (it.next()) ++yielded;
  } catch (const mtbl::Panic&) { panicked = true; }
  CHECK(panicked && yielded == 0);
  // the same file read with verify_checksums(false) does not panic on the checksum
  const mtbl::Reader r2 = mtbl::ReaderBuilder().verify_checksums(false).read(good);
  CHECK(r2.len() == 2000);
}

int main() {
  test_empty();
  test_one_key();
  test_separator_short();
  test_out_of_order();
  test_cfg1(mtbl::CompressionType::None);
  test_cfg1(mtbl::CompressionType::Snappy);
  test_errors();
  test_seek_kat();
  std::printf("OK %d\n", g_checks);
  return 0;
}
