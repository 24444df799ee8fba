"""Golden vectors for the transcript corruption of the data path:
the reference's CommonVoiceDataset.create_corrupted_transcript (trainer_unfreeze.py:784-829)
run on fixed texts under fixed `random` seeds -> corruption_golden.json (inputs + outputs only).

Run only in the build container (needs /root/reference):
    python tests/golden/make_corruption_golden.py
"""
import json
import random
from pathlib import Path

from make_golden import import_reference

HERE = Path(__file__).resolve().parent
TEXTS = [
    "o gato subiu no telhado ontem à noite",
    "eu gostaria de um café por favor",
    "sim",
    "",
    "duas palavras",
    "três palavras aqui",
    "uma frase bastante longa com muitas palavras para testar todas as estratégias de corrupção",
    "não sei",
]


def main():
    T = import_reference()
    corrupt = T.CommonVoiceDataset.create_corrupted_transcript
    cases = []
    for seed in range(40):
        for text in TEXTS:
            random.seed(seed)
            out = corrupt(None, text)
            cases.append({"seed": seed, "text": text, "out": out, "next_random": random.random()})
    (HERE / "corruption_golden.json").write_text(json.dumps({"source": "trainer_unfreeze.py:784-829",
                                                             "cases": cases}, ensure_ascii=False, indent=0))
    print(len(cases), "cases")


if __name__ == "__main__":
    main()
