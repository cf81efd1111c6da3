// storb_piece.hpp -- C++ host mirror of Storb's piece codec and of the
// zfec-rs API it calls, running on the MI355X path (include/storb_rs.h).
//
// The reference is Rust (crates/storb_base/src/piece.rs); there is no Rust
// toolchain in this build, so the host layer above the C ABI is C++ and
// keeps the reference's names, argument meaning and error behaviour:
//
//   storb::zfec::Fec / Chunk            zfec-rs @3f3a3720 as used at
//                                       piece.rs:9,328-329,375,383-386
//   storb::piece::piece_length          piece.rs:292-303
//   storb::piece::get_k_and_m           piece.rs:307-317
//   storb::piece::encode_chunk          piece.rs:320-361
//   storb::piece::decode_chunk          piece.rs:363-387
//   storb::piece::reconstruct_data      piece.rs:389-438
//   storb::piece::reconstruct_chunk     piece.rs:441-481
//   Piece / PieceType / EncodedChunk / PieceError   piece.rs:157-213
//
// Rust `.expect(..)` panics become a thrown storb::Panic; Rust Result<T, E>
// becomes storb::Result<T, E>. Every call runs on a per-thread context
// whose GPU is picked round-robin (objects partition across devices).
#pragma once

#include <cstdint>
#include <array>
#include <optional>
#include <stdexcept>
#include <string>
#include <utility>
#include <variant>
#include <vector>

struct storb_rs_ctx;

namespace storb {

struct Panic : std::runtime_error {
  using std::runtime_error::runtime_error;
};

template <class T, class E>
class Result {
 public:
  static Result Ok(T v) { return Result(std::move(v)); }
  static Result Err(E e) { return Result(std::move(e), 0); }
  bool is_ok() const { return v_.index() == 0; }
  bool is_err() const { return !is_ok(); }
  T &value() { return std::get<0>(v_); }
  const T &value() const { return std::get<0>(v_); }
  const E &error() const { return std::get<1>(v_); }
  // Rust `.expect(msg)`: the value, or panic.
  T expect(const std::string &msg) && {
    if (is_err()) throw Panic(msg + ": " + error().what());
    return std::move(std::get<0>(v_));
  }

 private:
  explicit Result(T v) : v_(std::in_place_index<0>, std::move(v)) {}
  Result(E e, int) : v_(std::in_place_index<1>, std::move(e)) {}
  std::variant<T, E> v_;
};

// The thread's MI355X context (created on first use, destroyed at thread
// exit). Throws storb::Panic when no gfx950 device is usable.
storb_rs_ctx *thread_ctx();

namespace zfec {

struct Error {
  int code = 0;
  std::string message;
  std::string what() const { return message; }
};

struct Chunk {
  std::vector<uint8_t> data;
  size_t index = 0;
  Chunk() = default;
  Chunk(std::vector<uint8_t> d, size_t i) : data(std::move(d)), index(i) {}
};

class Fec {
 public:
  // Fec::new(k, m): m is the TOTAL share count; k < 1, m < 1, m > 256 and
  // k > m are errors.
  static Result<Fec, Error> create(size_t k, size_t m);
  // Fec::encode: all m shares in index order (k zero-padded data shares,
  // m - k parity shares computed on the GPU) and the padding length.
  Result<std::pair<std::vector<Chunk>, size_t>, Error> encode(const uint8_t *data,
                                                               size_t len) const;
  Result<std::pair<std::vector<Chunk>, size_t>, Error> encode(
      const std::vector<uint8_t> &data) const {
    return encode(data.data(), data.size());
  }
  // Fec::decode: the data (k*B - padding bytes) from >= k shares.
  Result<std::vector<uint8_t>, Error> decode(const std::vector<Chunk> &chunks,
                                             size_t padding) const;
  size_t k() const { return k_; }
  size_t m() const { return m_; }

 private:
  Fec(size_t k, size_t m) : k_(k), m_(m) {}
  size_t k_, m_;
};

}  // namespace zfec

namespace piece {

enum class PieceType : uint8_t { Data = 0, Parity = 1 };

// TryFrom<u8> (piece.rs:172-182).
Result<PieceType, std::runtime_error> piece_type_from_u8(uint8_t v);

struct Piece {
  uint64_t chunk_idx = 0;
  uint64_t piece_size = 0;  // piece_length(chunk len), not data.size()
  uint64_t piece_idx = 0;
  PieceType piece_type = PieceType::Data;
  std::vector<uint8_t> data;
};

struct EncodedChunk {
  std::vector<Piece> pieces;
  uint64_t chunk_idx = 0;
  uint64_t k = 0;  // number of data blocks
  uint64_t m = 0;  // total blocks (data + parity)
  uint64_t chunk_size = 0;  // B = div_ceil(len, k)
  uint64_t padlen = 0;
  uint64_t original_chunk_size = 0;
};

struct PieceError {
  // ReconstructionError(chunk_idx, k, got)
  uint64_t chunk_idx = 0;
  uint64_t k = 0;
  size_t got = 0;
  std::string what() const;
};

uint64_t piece_length(uint64_t content_length,
                      std::optional<uint64_t> min_size = std::nullopt,
                      std::optional<uint64_t> max_size = std::nullopt);
std::pair<size_t, size_t> get_k_and_m(uint64_t chunk_size);

EncodedChunk encode_chunk(const uint8_t *chunk, size_t len, uint64_t chunk_idx);
inline EncodedChunk encode_chunk(const std::vector<uint8_t> &chunk, uint64_t chunk_idx) {
  return encode_chunk(chunk.data(), chunk.size(), chunk_idx);
}
std::vector<uint8_t> decode_chunk(const EncodedChunk &encoded_chunk);
std::vector<uint8_t> reconstruct_data(const std::vector<Piece> &pieces,
                                      const std::vector<EncodedChunk> &chunks);
Result<std::vector<uint8_t>, PieceError> reconstruct_chunk(const EncodedChunk &chunk);

// piece.rs:257-276: blake3(owner account id || piece hashes...), the
// object's InfoHash (upload.rs:292). 32-byte hashes in, 32 bytes out.
std::array<uint8_t, 32> get_infohash_by_identity(
    const std::vector<std::array<uint8_t, 32>> &piece_hashes,
    const std::vector<uint8_t> &owner_account_id);

}  // namespace piece
}  // namespace storb
