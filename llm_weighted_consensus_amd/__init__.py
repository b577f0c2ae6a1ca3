"""llm_weighted_consensus_amd — an MI355X-native weighted-consensus LLM server.

Same capabilities and wire API as ObjectiveAI/llm-weighted-consensus (OpenAI-compatible
/chat/completions and /score/completions with weighted LLM voters, completions archive, multichat and
embeddings types), but generation, embeddings and scoring run in-process on AMD MI355X (gfx950) with
hand-written HIP kernels, and multi-GPU work goes over RCCL/xGMI.

Sub-packages:
  schema/    wire types + streaming merge algebra       score/    voters, key tree, votes, tally, ids
  chat/      chat clients (local engine, remote, fake) archive/  completions archive + reference resolution
  engine/    paged-KV continuous-batching engine        models/   Llama / Mixtral decoders, BERT encoders
  ops/       gfx950 HIP kernels (torch bindings)        parallel/ torch.distributed (RCCL) bring-up, collectives
  embeddings/ embedding service + consensus scorer      server/   config + ASGI app (SSE)
  utils/     canonical JSON, ids, misc
"""
__version__ = "0.1.0"
