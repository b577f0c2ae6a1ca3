#include "block_manager.h"

#include <string>

namespace lwc {

BlockManager::BlockManager(int num_blocks, int block_size) : num_blocks_(num_blocks), block_size_(block_size) {
  if (num_blocks <= 0 || block_size <= 0) throw std::invalid_argument("BlockManager: sizes must be positive");
  free_.reserve(num_blocks);
  // pop_back() hands out low block ids first
  for (int b = num_blocks - 1; b >= 0; --b) free_.push_back(b);
  ref_.assign(num_blocks, 0);
}

const BlockManager::Seq& BlockManager::get(int64_t seq) const {
  auto it = seqs_.find(seq);
  if (it == seqs_.end()) throw std::out_of_range("BlockManager: unknown sequence " + std::to_string(seq));
  return it->second;
}
BlockManager::Seq& BlockManager::get(int64_t seq) {
  auto it = seqs_.find(seq);
  if (it == seqs_.end()) throw std::out_of_range("BlockManager: unknown sequence " + std::to_string(seq));
  return it->second;
}

int32_t BlockManager::alloc_block() {
  if (free_.empty()) throw std::runtime_error("BlockManager: out of KV blocks");
  const int32_t b = free_.back();
  free_.pop_back();
  ref_[b] = 1;
  return b;
}

void BlockManager::release(int32_t block) {
  if (ref_[block] <= 0) throw std::logic_error("BlockManager: double free of block " + std::to_string(block));
  if (--ref_[block] == 0) free_.push_back(block);
}

void BlockManager::add_sequence(int64_t seq, int64_t num_tokens) {
  if (seqs_.count(seq)) throw std::invalid_argument("BlockManager: sequence exists " + std::to_string(seq));
  const int need = blocks_for(num_tokens);
  if (!can_allocate(need)) throw std::runtime_error("BlockManager: out of KV blocks");
  Seq s;
  s.blocks.reserve(need + 8);
  for (int i = 0; i < need; ++i) s.blocks.push_back(alloc_block());
  s.len = num_tokens;
  seqs_.emplace(seq, std::move(s));
}

void BlockManager::fork(int64_t parent, int64_t child) {
  if (seqs_.count(child)) throw std::invalid_argument("BlockManager: sequence exists " + std::to_string(child));
  const Seq& p = get(parent);
  Seq c;
  c.blocks = p.blocks;
  c.len = p.len;
  for (int32_t b : c.blocks) ++ref_[b];
  seqs_.emplace(child, std::move(c));
}

int BlockManager::append_cost(int64_t seq) const {
  const Seq& s = get(seq);
  if (s.len % block_size_ == 0) return 1;          // needs a fresh block
  return ref_[s.blocks.back()] > 1 ? 1 : 0;         // copy-on-write of a shared partial block
}

int64_t BlockManager::append_token(int64_t seq) {
  Seq& s = get(seq);
  const int64_t pos = s.len;
  if (pos % block_size_ == 0) {
    s.blocks.push_back(alloc_block());
  } else {
    int32_t& last = s.blocks.back();
    if (ref_[last] > 1) {  // copy-on-write
      const int32_t nb = alloc_block();
      copies_.emplace_back(last, nb);
      --ref_[last];
      last = nb;
    }
  }
  s.len = pos + 1;
  return (int64_t)s.blocks[pos / block_size_] * block_size_ + pos % block_size_;
}

int64_t BlockManager::slot(int64_t seq, int64_t pos) const {
  const Seq& s = get(seq);
  if (pos < 0 || pos >= s.len) throw std::out_of_range("BlockManager: position out of range");
  return (int64_t)s.blocks[pos / block_size_] * block_size_ + pos % block_size_;
}

void BlockManager::free_sequence(int64_t seq) {
  auto it = seqs_.find(seq);
  if (it == seqs_.end()) return;
  for (int32_t b : it->second.blocks) release(b);
  seqs_.erase(it);
}

std::vector<std::pair<int32_t, int32_t>> BlockManager::take_copies() {
  std::vector<std::pair<int32_t, int32_t>> out;
  out.swap(copies_);
  return out;
}

}  // namespace lwc
