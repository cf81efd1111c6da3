// piece.cpp -- C++ host mirror of crates/storb_base/src/piece.rs and of the
// zfec-rs calls it makes, over the C ABI of include/storb_rs.h.
#include "../../include/storb_piece.hpp"

#include <algorithm>
#include <memory>

#include "../../include/storb_rs.h"

namespace storb {

namespace {

struct CtxHolder {
  storb_rs_ctx *ctx = nullptr;
  ~CtxHolder() {
    if (ctx) storb_rs_ctx_destroy(ctx);
  }
};

}  // namespace

storb_rs_ctx *thread_ctx() {
  thread_local CtxHolder h;
  if (!h.ctx) {
    const int rc = storb_rs_ctx_create(-1, &h.ctx);
    if (rc != STORB_RS_OK)
      throw Panic(std::string("storb_rs_ctx_create: ") + storb_rs_strerror(rc));
  }
  return h.ctx;
}

namespace zfec {

namespace {
Error make_error(int code) {
  std::string msg = storb_rs_strerror(code);
  if (code == STORB_RS_EDEVICE || code == STORB_RS_ENOMEM) {
    const char *d = storb_rs_last_error(thread_ctx());
    if (d && *d) msg += std::string(" (") + d + ")";
  }
  return Error{code, msg};
}
}  // namespace

Result<Fec, Error> Fec::create(size_t k, size_t m) {
  if (k > STORB_RS_MAX_SHARES || m > STORB_RS_MAX_SHARES ||
      storb_rs_check_params(static_cast<uint32_t>(k), static_cast<uint32_t>(m)) !=
          STORB_RS_OK)
    return Result<Fec, Error>::Err(Error{STORB_RS_EINVAL, "invalid (k, m)"});
  return Result<Fec, Error>::Ok(Fec(k, m));
}

Result<std::pair<std::vector<Chunk>, size_t>, Error> Fec::encode(const uint8_t *data,
                                                                 size_t len) const {
  using R = Result<std::pair<std::vector<Chunk>, size_t>, Error>;
  const uint32_t k = static_cast<uint32_t>(k_), n = static_cast<uint32_t>(m_);
  if (len == 0) return R::Err(Error{STORB_RS_EINVAL, "empty input"});
  const size_t B = storb_rs_block_size(k, len);
  std::vector<Chunk> chunks(n);
  for (uint32_t i = 0; i < n; i++) {
    chunks[i].index = i;
    chunks[i].data.assign(B, 0);
  }
  // Systematic: data shares are the zero-padded slices of the input.
  for (uint32_t j = 0; j < k; j++) {
    const size_t off = static_cast<size_t>(j) * B;
    if (off < len)
      std::copy(data + off, data + off + std::min(B, len - off), chunks[j].data.begin());
  }
  size_t block = 0, pad = 0;
  std::vector<uint8_t *> parity(n - k);
  for (uint32_t i = k; i < n; i++) parity[i - k] = chunks[i].data.data();
  const int rc =
      storb_rs_encode(thread_ctx(), k, n, data, len, parity.data(), &block, &pad);
  if (rc != STORB_RS_OK) return R::Err(make_error(rc));
  return R::Ok(std::make_pair(std::move(chunks), pad));
}

Result<std::vector<uint8_t>, Error> Fec::decode(const std::vector<Chunk> &chunks,
                                                size_t padding) const {
  using R = Result<std::vector<uint8_t>, Error>;
  const uint32_t k = static_cast<uint32_t>(k_), n = static_cast<uint32_t>(m_);
  if (chunks.size() < k) return R::Err(make_error(STORB_RS_ENOTENOUGH));
  const size_t B = chunks[0].data.size();
  std::vector<const uint8_t *> ptrs;
  std::vector<uint32_t> idx;
  for (const Chunk &c : chunks) {
    if (c.data.size() != B)
      return R::Err(Error{STORB_RS_EINVAL, "shares of different lengths"});
    if (c.index >= n) return R::Err(Error{STORB_RS_EINVAL, "share index >= m"});
    ptrs.push_back(c.data.data());
    idx.push_back(static_cast<uint32_t>(c.index));
  }
  if (B == 0 || padding >= static_cast<size_t>(k) * B)
    return R::Err(Error{STORB_RS_EINVAL, "bad padding / empty shares"});
  std::vector<uint8_t> out(static_cast<size_t>(k) * B - padding);
  const int rc = storb_rs_decode(thread_ctx(), k, n, ptrs.data(), idx.data(),
                                 static_cast<uint32_t>(idx.size()), B, padding, out.data());
  if (rc != STORB_RS_OK) return R::Err(make_error(rc));
  return R::Ok(std::move(out));
}

}  // namespace zfec

namespace piece {

Result<PieceType, std::runtime_error> piece_type_from_u8(uint8_t v) {
  using R = Result<PieceType, std::runtime_error>;
  if (v == 0) return R::Ok(PieceType::Data);
  if (v == 1) return R::Ok(PieceType::Parity);
  return R::Err(std::runtime_error("Invalid PieceType value"));
}

std::string PieceError::what() const {
  return "Not enough pieces to reconstruct chunk " + std::to_string(chunk_idx) +
         ", expected k=" + std::to_string(k) + " but got " + std::to_string(got) +
         " pieces";
}

uint64_t piece_length(uint64_t content_length, std::optional<uint64_t> min_size,
                      std::optional<uint64_t> max_size) {
  const uint64_t lo = min_size.value_or(16ull * 1024);
  const uint64_t hi = max_size.value_or(256ull * 1024 * 1024);
  // storb_piece_length treats 0 as "default"; Rust clamp(lo, hi) with an
  // explicit 0 bound only matters for min_size = 0 (no lower clamp).
  uint64_t v = storb_piece_length(content_length, 1, UINT64_MAX);
  return std::min(std::max(v, lo), hi);
}

std::pair<size_t, size_t> get_k_and_m(uint64_t chunk_size) {
  uint64_t k = 0, m = 0;
  storb_get_k_and_m(chunk_size, &k, &m);
  return {static_cast<size_t>(k), static_cast<size_t>(m)};
}

EncodedChunk encode_chunk(const uint8_t *chunk, size_t len, uint64_t chunk_idx) {
  const uint64_t chunk_size = len;
  const uint64_t piece_size = piece_length(chunk_size);
  const auto [k, m] = get_k_and_m(chunk_size);
  zfec::Fec encoder = zfec::Fec::create(k, m).expect("Failed to create encoder");
  auto enc = encoder.encode(chunk, len).expect("Failed to encode chunk");
  const uint64_t zfec_chunk_size = (chunk_size + k - 1) / k;  // piece.rs:331-332
  EncodedChunk out;
  out.pieces.reserve(enc.first.size());
  for (size_t i = 0; i < enc.first.size(); i++) {
    Piece p;
    p.piece_type = i < k ? PieceType::Data : PieceType::Parity;
    p.piece_size = piece_size;
    p.data = std::move(enc.first[i].data);
    p.chunk_idx = chunk_idx;
    p.piece_idx = i;
    out.pieces.push_back(std::move(p));
  }
  out.chunk_idx = chunk_idx;
  out.k = k;
  out.m = m;
  out.chunk_size = zfec_chunk_size;
  out.padlen = enc.second;
  out.original_chunk_size = chunk_size;
  return out;
}

std::vector<uint8_t> decode_chunk(const EncodedChunk &encoded_chunk) {
  const size_t k = encoded_chunk.k, m = encoded_chunk.m;
  std::vector<const Piece *> pieces;
  for (const Piece &p : encoded_chunk.pieces) pieces.push_back(&p);
  std::stable_sort(pieces.begin(), pieces.end(),
                   [](const Piece *a, const Piece *b) { return a->piece_idx < b->piece_idx; });
  // zfec decode requires exactly k blocks (piece.rs:371-381)
  if (pieces.size() > k) pieces.resize(k);
  std::vector<zfec::Chunk> to_decode;
  for (const Piece *p : pieces) to_decode.emplace_back(p->data, p->piece_idx);
  zfec::Fec decoder = zfec::Fec::create(k, m).expect("Failed to create decoder");
  return decoder.decode(to_decode, encoded_chunk.padlen).expect("Failed to decode chunk");
}

std::vector<uint8_t> reconstruct_data(const std::vector<Piece> &pieces,
                                      const std::vector<EncodedChunk> &chunks) {
  std::vector<uint8_t> out;
  for (const EncodedChunk &chunk : chunks) {
    std::vector<Piece> relevant;
    for (const Piece &p : pieces)
      if (p.chunk_idx == chunk.chunk_idx) relevant.push_back(p);
    std::stable_sort(relevant.begin(), relevant.end(),
                     [](const Piece &a, const Piece &b) { return a.piece_idx < b.piece_idx; });
    if (relevant.size() < chunk.k) return {};  // piece.rs:411-421: empty = error
    EncodedChunk to_decode = chunk;
    to_decode.pieces = std::move(relevant);
    std::vector<uint8_t> part = decode_chunk(to_decode);
    out.insert(out.end(), part.begin(), part.end());
  }
  return out;
}

Result<std::vector<uint8_t>, PieceError> reconstruct_chunk(const EncodedChunk &chunk) {
  using R = Result<std::vector<uint8_t>, PieceError>;
  std::vector<Piece> relevant;
  for (const Piece &p : chunk.pieces)
    if (p.chunk_idx == chunk.chunk_idx) relevant.push_back(p);
  std::stable_sort(relevant.begin(), relevant.end(),
                   [](const Piece &a, const Piece &b) { return a.piece_idx < b.piece_idx; });
  if (relevant.size() < chunk.k)
    return R::Err(PieceError{chunk.chunk_idx, chunk.k, relevant.size()});
  EncodedChunk to_decode = chunk;
  to_decode.pieces = std::move(relevant);
  return R::Ok(decode_chunk(to_decode));
}

std::array<uint8_t, 32> get_infohash_by_identity(
    const std::vector<std::array<uint8_t, 32>> &piece_hashes,
    const std::vector<uint8_t> &owner_account_id) {
  std::vector<uint8_t> msg(owner_account_id);
  for (const auto &h : piece_hashes) msg.insert(msg.end(), h.begin(), h.end());
  std::array<uint8_t, 32> out{};
  storb_blake3(msg.data(), msg.size(), out.data());
  return out;
}

}  // namespace piece
}  // namespace storb
