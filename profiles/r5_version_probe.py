"""Which parameters' tensor versions move between optimizer steps (each one makes
ParamStore.sync_shadow re-cast its bf16 shadow at the next step: 205 cast_kernel launches per c2
step in profiles/r5d's kernel stats)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from speech_transcript_embeddings_amd.model import EnhancedAudioTextModel  # noqa: E402
from speech_transcript_embeddings_amd.train import TrainStep, synthetic_batch  # noqa: E402

model = EnhancedAudioTextModel(device="cuda:0", spec_augment=False)
model.audio_cfg.layerdrop = 0.0
step = TrainStep(model, warmup=100, total_steps=1000, micro_batch=2, max_text_length=16)
data = synthetic_batch(2, 32000, 16, device="cuda:0")
st = model.store
calls = []
orig = st.sync_shadow


def spy(force=False):
    stale = [n for n in st.slots if force or st._versions.get(n) != st.params[n]._version]
    calls.append(stale)
    return orig(force)


st.sync_shadow = spy
for _ in range(3):
    step(*data)
torch.cuda.synchronize()
for i, c in enumerate(calls):
    print(f"step {i}: {len(c)} stale shadows; first: {c[:6]}")
