"""MI355X-native speech<->transcript contrastive training step.

A from-scratch gfx950 implementation of the hot path of
yuriyvnv/speech_transcript_embeddings (training/trainer_unfreeze.py:train_epoch):
GPU fbank -> w2v-bert Conformer + XLM-R encoders -> pooling / projection /
cross-modal heads -> AlignmentAwareInfoNCE -> backward -> clip -> AdamW, with
every hot op a hand-written HIP kernel in libste.so (include/ste.h).
"""
__version__ = "0.2.0"

from . import torch_ops  # noqa: E402,F401  (torch.ops.ste.* custom operators)
