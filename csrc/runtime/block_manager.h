// Paged-KV block manager for the MI355X engine (host side, C++).
//
// The KV cache of every GPU is one flat pool of fixed-size blocks (BS tokens x all layers).  A
// sequence owns an ordered block table; blocks are reference counted so a sequence can be FORKED
// (the N candidates / voters of one request share their prompt's blocks) and the first write into a
// shared block triggers copy-on-write: a fresh block is allocated and a (src, dst) copy is queued
// for the GPU (kv_block_copy kernel, K12) before the step that writes it.
//
// Sized for 288 GB of HBM3E: block ids are int32 (2^31 blocks x 16 tokens), sequence ids int64.
#pragma once
#include <cstdint>
#include <list>
#include <stdexcept>
#include <unordered_map>
#include <utility>
#include <vector>

namespace lwc {

class BlockManager {
 public:
  BlockManager(int num_blocks, int block_size);

  int num_blocks() const { return num_blocks_; }
  int block_size() const { return block_size_; }
  // free blocks + unreferenced prefix-cache blocks (reclaimed on demand, least recently used first)
  int num_free() const { return (int)(free_.size() + lru_.size()); }
  int num_sequences() const { return (int)seqs_.size(); }
  bool has_sequence(int64_t seq) const { return seqs_.count(seq) != 0; }

  // Blocks needed to hold `num_tokens` tokens for a new sequence.
  int blocks_for(int64_t num_tokens) const { return (int)((num_tokens + block_size_ - 1) / block_size_); }
  bool can_allocate(int num_blocks) const { return num_free() >= num_blocks; }

  // Allocate a new sequence able to hold `num_tokens` tokens (its length is set to num_tokens).
  void add_sequence(int64_t seq, int64_t num_tokens);
  // Child shares every block of the parent (refcount++), same length.
  void fork(int64_t parent, int64_t child);
  // Grow the sequence by one token; returns the cache slot (block*BS + offset) of that token.
  // Allocates a new block at block boundaries and performs copy-on-write on a shared last block.
  int64_t append_token(int64_t seq);
  // Number of extra blocks `append_token` may need for this sequence (0 or 1).
  int append_cost(int64_t seq) const;
  void free_sequence(int64_t seq);

  int64_t length(int64_t seq) const { return get(seq).len; }
  const std::vector<int32_t>& block_table(int64_t seq) const { return get(seq).blocks; }
  // Slot of token position `pos` of the sequence.
  int64_t slot(int64_t seq, int64_t pos) const;
  int refcount(int32_t block) const { return ref_[block]; }

  // Extra blocks one append_token on each of `seqs` may need (upper bound: every sharer of a shared
  // partial last block is counted as a copy-on-write).
  int64_t append_cost_total(const std::vector<int64_t>& seqs) const;

  // ---- preemption by swapping (exact: the KV bytes leave and come back unchanged) ----
  // A group of sequences (forked: they share blocks) is exported as its distinct blocks in first-use
  // order plus, per sequence, its table as indices into that list; the sequences are then freed.  The
  // caller copies the listed blocks' KV out BEFORE any later work can reuse them (stream order).
  struct Swapped {
    std::vector<int32_t> blocks;                 // distinct physical blocks, first-use order
    std::vector<std::vector<int32_t>> tables;    // per sequence: indices into `blocks`
    std::vector<int64_t> lens;
  };
  Swapped swap_out(const std::vector<int64_t>& seqs);
  // Re-create the sequences on `n` fresh blocks with the exported structure (shared blocks shared again,
  // refcount = number of referencing sequences); returns the new physical block of each exported index.
  std::vector<int32_t> swap_in(const std::vector<int64_t>& seqs, int n, const std::vector<std::vector<int32_t>>& tables,
                               const std::vector<int64_t>& lens);

  // Copy-on-write copies queued since the last call (src, dst); cleared by this call.
  std::vector<std::pair<int32_t, int32_t>> take_copies();

  // ---- automatic prefix caching (cross-request KV reuse) ----
  // A FULL prompt block can be registered under a chain key: key_i = H(key_{i-1}, the block's BS token
  // ids), key_{-1} = a root constant, so a key names the whole token prefix up to that block.  A later
  // sequence whose prompt starts with the same tokens takes those blocks by reference instead of
  // recomputing them; every match also compares the block's stored tokens and parent key.  Registered
  // blocks that no sequence references stay resident in an LRU list and are reclaimed only when the pool
  // runs dry, so the cache costs no capacity.  Disabled by default.
  void set_prefix_caching(bool on);
  bool prefix_caching() const { return prefix_caching_; }
  // Prompt tokens a new sequence would take from the cache: a multiple of BS, and at most
  // tokens.size() - 1 (the last prompt token is always computed: its logits start decoding).
  int64_t match_prefix(const std::vector<int32_t>& tokens) const;
  // add_sequence(seq, tokens.size()) reusing the cached prefix blocks; returns the reused token count.
  int64_t add_sequence_cached(int64_t seq, const std::vector<int32_t>& tokens);
  // Register the sequence's blocks that `tokens` (its prompt) fills completely.
  void cache_prefix(int64_t seq, const std::vector<int32_t>& tokens);
  int num_cached_blocks() const { return (int)by_key_.size(); }
  int num_evictable() const { return (int)lru_.size(); }

 private:
  struct Seq {
    std::vector<int32_t> blocks;
    int64_t len = 0;
  };
  const Seq& get(int64_t seq) const;
  Seq& get(int64_t seq);
  int32_t alloc_block();
  void release(int32_t block);
  void acquire_cached(int32_t block);
  void unregister(int32_t block);
  uint64_t chain_key(uint64_t parent, const int32_t* toks) const;
  // walk the cached chain of `tokens`; returns matched block ids (<= max_blocks of them)
  std::vector<int32_t> match_blocks(const std::vector<int32_t>& tokens, int64_t max_blocks) const;

  int num_blocks_, block_size_;
  std::vector<int32_t> free_;
  std::vector<int32_t> ref_;
  // prefix cache
  bool prefix_caching_ = false;
  std::unordered_map<uint64_t, int32_t> by_key_;
  std::vector<uint64_t> key_, parent_key_;       // per block (valid when registered_[b])
  std::vector<char> registered_;
  std::vector<int32_t> block_tokens_;            // [num_blocks * BS] token ids of registered blocks
  std::list<int32_t> lru_;                       // unreferenced registered blocks, oldest first
  std::vector<std::list<int32_t>::iterator> lru_pos_;
  std::unordered_map<int64_t, Seq> seqs_;
  std::vector<std::pair<int32_t, int32_t>> copies_;
};

}  // namespace lwc
