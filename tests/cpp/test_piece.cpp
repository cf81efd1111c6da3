// test_piece.cpp -- the reference's piece.rs tests (piece.rs:506-689) ported
// onto the C++ host mirror (include/storb_piece.hpp), running on MI355X.
// The two erasure tests actually drop pieces here (the Rust versions drop
// nothing). Also: Appendix-B KATs through zfec::Fec, and
// concurrent encodes from several threads (one context per thread).
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "../../include/storb_piece.hpp"

using namespace storb;
using namespace storb::piece;

static int g_fail = 0;
#define CHECK(c)                                                   \
  do {                                                             \
    if (!(c)) {                                                    \
      std::fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #c); \
      g_fail++;                                                    \
    }                                                              \
  } while (0)

static std::vector<uint8_t> random_bytes(size_t n, uint64_t seed) {
  std::mt19937_64 g(seed);
  std::vector<uint8_t> v(n);
  for (auto &b : v) b = static_cast<uint8_t>(g());
  return v;
}

static std::vector<uint8_t> bytes_of(const char *s) {
  return std::vector<uint8_t>(s, s + std::string(s).size());
}

static std::vector<std::vector<uint8_t>> split(const std::vector<uint8_t> &d) {
  const size_t cs = piece_length(d.size());
  std::vector<std::vector<uint8_t>> out;
  for (size_t i = 0; i < d.size(); i += cs)
    out.emplace_back(d.begin() + i, d.begin() + std::min(d.size(), i + cs));
  return out;
}

static void test_piece_length() {
  CHECK(piece_length(1000) >= 16 * 1024);
  CHECK(piece_length(1000000) <= 256ull * 1024 * 1024);
}

static void test_encode_decode_chunk() {
  auto d = bytes_of("Hello, World!");
  auto enc = encode_chunk(d, 0);
  CHECK(decode_chunk(enc) == d);
}

static void test_encode_chunk_pieces() {
  auto enc = encode_chunk(bytes_of("Test data"), 0);
  size_t nd = 0, np = 0;
  for (auto &p : enc.pieces) (p.piece_type == PieceType::Data ? nd : np)++;
  CHECK(nd > 0 && np > 0);
}

static void test_reconstruct_data() {
  auto d = bytes_of("Test reconstruction");
  auto enc = encode_chunk(d, 0);
  CHECK(reconstruct_data(enc.pieces, {enc}) == d);
}

static void test_split_data() {
  const size_t size = 1 << 20;
  auto d = random_bytes(size, 1);
  size_t expected = 0, got = 0, nchunks = 0;
  auto parts = split(d);
  for (size_t i = 0; i < parts.size(); i++) {
    auto info = encode_chunk(parts[i], i);
    const uint64_t ps = piece_length(info.original_chunk_size);
    expected += info.m * ((info.chunk_size + ps - 1) / ps);
    got += info.pieces.size();
    nchunks++;
  }
  CHECK(nchunks == (size + piece_length(size) - 1) / piece_length(size));
  CHECK(got == expected);
}

static void test_reconstruct_data_large_and_corrupted() {
  const size_t size = 1 << 20;
  auto d = random_bytes(size, 2);
  std::mt19937 rng(7);
  std::vector<EncodedChunk> chunks;
  std::vector<Piece> all, kept;
  auto parts = split(d);
  for (size_t i = 0; i < parts.size(); i++) {
    auto info = encode_chunk(parts[i], i);
    chunks.push_back(info);
    all.insert(all.end(), info.pieces.begin(), info.pieces.end());
    auto ps = info.pieces;
    std::shuffle(ps.begin(), ps.end(), rng);
    ps.resize(static_cast<size_t>(std::ceil(ps.size() * 0.7)));
    kept.insert(kept.end(), ps.begin(), ps.end());
  }
  std::shuffle(all.begin(), all.end(), rng);
  std::shuffle(kept.begin(), kept.end(), rng);
  CHECK(reconstruct_data(all, chunks) == d);
  CHECK(reconstruct_data(kept, chunks) == d);
}

static void test_reconstruct_single_chunk() {
  std::vector<uint8_t> d(1024, 0);
  auto enc = encode_chunk(d, 0);
  auto r = reconstruct_chunk(enc);
  CHECK(r.is_ok() && r.value() == d);
  EncodedChunk reduced = enc;
  reduced.pieces.assign(enc.pieces.end() - enc.k, enc.pieces.end());
  auto r2 = reconstruct_chunk(reduced);
  CHECK(r2.is_ok() && r2.value() == d);
  EncodedChunk few = enc;
  few.pieces.assign(enc.pieces.begin(), enc.pieces.begin() + (enc.k - 1));
  auto r3 = reconstruct_chunk(few);
  CHECK(r3.is_err());
  if (r3.is_err()) CHECK(r3.error().what().find("Not enough pieces") == 0);
}

static void test_fec_kats_appendix_b() {
  struct Kat {
    size_t k, n;
    std::vector<uint8_t> data;
    std::vector<std::vector<uint8_t>> parity;
  };
  std::vector<Kat> kats = {
      {4, 6, {1, 2, 3, 4}, {{0x87}, {0x2e}}},
      {4, 6, {0, 1, 2, 3, 4, 5, 6, 7, 8, 9}, {{0x2e, 0xc2, 0x6e}, {0xf1, 0x42, 0xfa}}},
      {8, 12, {1, 2, 3, 4, 5, 6, 7, 8}, {{0x70}, {0x25}, {0xe1}, {0x6e}}},
      {2, 3, bytes_of("Test data"), {{0x34, 0x6d, 0x7d, 0x5e, 0x60}}},
  };
  for (auto &t : kats) {
    auto fec = zfec::Fec::create(t.k, t.n).expect("create");
    auto enc = fec.encode(t.data).expect("encode");
    for (size_t i = 0; i < t.parity.size(); i++) CHECK(enc.first[t.k + i].data == t.parity[i]);
    // decode through parity only where possible
    std::vector<zfec::Chunk> sub(enc.first.end() - t.k, enc.first.end());
    auto dec = fec.decode(sub, enc.second).expect("decode");
    CHECK(dec == t.data);
  }
  CHECK(zfec::Fec::create(0, 2).is_err());
  CHECK(zfec::Fec::create(3, 2).is_err());
  CHECK(zfec::Fec::create(2, 257).is_err());
  bool panicked = false;
  try {
    encode_chunk(std::vector<uint8_t>{}, 0);  // k = 0: Fec::new fails -> panic
  } catch (const Panic &) {
    panicked = true;
  }
  CHECK(panicked);
}

static void test_threads() {
  std::vector<std::thread> ts;
  std::vector<int> ok(4, 0);
  for (int t = 0; t < 4; t++)
    ts.emplace_back([t, &ok] {
      auto d = random_bytes((3u << 20) + 1234 * t, 50 + t);
      auto enc = encode_chunk(d, t);
      auto keep = enc.pieces;
      keep.erase(keep.begin(), keep.begin() + std::min<size_t>(enc.m - enc.k, enc.k));
      EncodedChunk c = enc;
      c.pieces = keep;
      auto r = reconstruct_chunk(c);
      ok[t] = r.is_ok() && r.value() == d;
    });
  for (auto &t : ts) t.join();
  for (int v : ok) CHECK(v == 1);
}

// get_infohash_by_identity (piece.rs:257-276) on a fixed input; the expected
// digest is blake3(owner || hashes) from the restated reference
// (oracle/blake3_ref.py), itself pinned to the published vectors.
static void test_infohash() {
  std::vector<uint8_t> owner(32);
  for (int i = 0; i < 32; i++) owner[i] = static_cast<uint8_t>(i);
  std::vector<std::array<uint8_t, 32>> hs(3);
  for (int i = 0; i < 3; i++) hs[i].fill(static_cast<uint8_t>(i));
  const auto got = get_infohash_by_identity(hs, owner);
  static const char *want = "2efb6fabb62a24e9d0690fb306c6ba2c234085b6352c1e41cc981d075caffa2d";
  char hex[65];
  for (int i = 0; i < 32; i++) std::snprintf(hex + 2 * i, 3, "%02x", got[i]);
  CHECK(std::string(hex) == want);
}

int main() {
  test_piece_length();
  test_encode_decode_chunk();
  test_encode_chunk_pieces();
  test_reconstruct_data();
  test_split_data();
  test_reconstruct_data_large_and_corrupted();
  test_reconstruct_single_chunk();
  test_fec_kats_appendix_b();
  test_threads();
  test_infohash();
  if (g_fail) {
    std::fprintf(stderr, "%d check(s) failed\n", g_fail);
    return 1;
  }
  std::printf("test_piece: all checks passed\n");
  return 0;
}
