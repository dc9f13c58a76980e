"""Golden output of BASELINE configs[0]: the reference's own examples/cli (whisper-cli), CPU
backend, 1 thread, on samples/jfk.wav, with the synthetic tiny.en model.

The reference CLI (ref examples/cli/cli.cpp + common sources) linked to the reference library is
built by oracle/ref/Makefile into oracle/_ref/whisper-cli. The same unchanged sources linked to
OUR libwhisper.so are built by `make callers` (open-whisper-kit_amd/lib/callers/whisper-cli);
tests/test_callers.py runs that one on the GPU and compares its full JSON output with this file.

Cases: the CLI defaults (beam 5 + best-of 5, temperature fallback; ref cli.cpp:45-84) and `-nf`
(no fallback), each as `-ojf` full JSON (segments, tokens with ids/p/t0/t1); and GBNF
grammar-constrained decoding (`--grammar <text> --grammar-rule root`, parsed by the reference's
examples/grammar-parser.cpp inside the CLI; beam search as the CLI selects it with a grammar,
ref cli.cpp:1170-1171, 1225-1238; constraint logic ref src/whisper.cpp:5498-5905): a word list
with alternation and repetition, and character classes with ranges and a negated class (the
latter ends on a partial UTF-8 byte token), without and with timestamps.

Usage (container with /root/reference):  python tests/golden/make_golden_cli.py
"""
import json
import os
import subprocess
import sys
import tempfile

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(ROOT, "open-whisper-kit_amd", "python"))
import owk_synth as S  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))
SEED = 1234
MODEL = "tiny.en"
GRAMMARS = {
    "words": 'root ::= (" " word ",")+ " " word "."\nword ::= "red" | "green" | "blue" | "yellow" | "purple"\n',
    "moves": 'root ::= move (" " move)* [^a-z0-9 ]\nmove ::= " "? [a-h] [1-8] | " castle"\n',
}
CASES = {"default": [], "nofallback": ["-nf"],
         "grammar_words": ["-nf", "-nt", "--grammar", GRAMMARS["words"], "--grammar-rule", "root"],
         "grammar_moves": ["-nf", "-nt", "--grammar", GRAMMARS["moves"], "--grammar-rule", "root", "--grammar-penalty", "50"],
         "grammar_words_ts": ["-nf", "--grammar", GRAMMARS["words"], "--grammar-rule", "root"]}


def run_cli(exe, model_path, wav, extra, workdir):
    """Run a whisper-cli binary; returns (exit code, parsed -ojf JSON or None)."""
    base = os.path.join(workdir, "out")
    if os.path.exists(base + ".json"):
        os.remove(base + ".json")
    cmd = [exe, "-m", model_path, "-f", wav, "-t", "1", "-np", "-ojf", "-of", base] + list(extra)
    r = subprocess.run(cmd, capture_output=True, text=True)
    doc = None
    if os.path.exists(base + ".json"):
        with open(base + ".json", encoding="utf-8", errors="replace") as f:
            doc = json.load(f)
    return r.returncode, doc


def comparable(doc):
    """The parts of the CLI JSON that depend on the engine's results (drops system info)."""
    return {"result": doc["result"], "transcription": doc["transcription"]}


def main():
    cache = os.environ.get("OWK_MODEL_CACHE", "/tmp/owk_models")
    os.makedirs(cache, exist_ok=True)
    path = os.path.join(cache, f"synth-{MODEL}-s{SEED}.bin")
    sha = S.write_model(path, MODEL, SEED)
    exe = os.path.join(ROOT, "oracle", "_ref", "whisper-cli")
    meta = {"seed": SEED, "model": MODEL, "sha256": sha, "wav": "jfk.wav", "cases": {}}
    with tempfile.TemporaryDirectory() as td:
        for name, extra in CASES.items():
            code, doc = run_cli(exe, path, os.path.join(OUT, "jfk.wav"), extra, td)
            assert code == 0 and doc is not None, (name, code)
            meta["cases"][name] = {"args": extra, "exit": code, "json": comparable(doc)}
            segs = doc["transcription"]
            print(name, len(segs), "segments", sum(len(s["tokens"]) for s in segs), "tokens")
    with open(os.path.join(OUT, "cli_golden.json"), "w") as f:
        json.dump(meta, f, indent=1)


if __name__ == "__main__":
    main()
