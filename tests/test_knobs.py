"""Build-time knobs of the shipped kernel sources (CPU only): every preprocessor
conditional in libpnet_amd/csrc/ names a macro of the allowlist in
csrc/rx_config.h (the kernel-shape parameters, each with its default there,
plus the PNET_WAVE_TIMES diagnostic build), and no other file defines a
default for one. Rejected A/B variants do not live in the product sources."""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "libpnet_amd", "csrc")
DIAGNOSTIC = {"PNET_WAVE_TIMES"}


def _sources():
    for f in sorted(os.listdir(CSRC)):
        if f.endswith((".h", ".hip", ".cpp")):
            yield f, open(os.path.join(CSRC, f)).read()


def _allowlist():
    text = open(os.path.join(CSRC, "rx_config.h")).read()
    return set(re.findall(r"^#ifndef (PNET\w*)$", text, re.M))


def test_allowlist_is_small_and_has_defaults():
    allow = _allowlist()
    assert 0 < len(allow | DIAGNOSTIC) <= 12, sorted(allow)
    text = open(os.path.join(CSRC, "rx_config.h")).read()
    for k in allow:
        assert re.search(rf"^#ifndef {k}\n#define {k} \S", text, re.M), k


def test_every_conditional_names_an_allowlisted_knob():
    allow = _allowlist() | DIAGNOSTIC
    for f, text in _sources():
        for line in re.findall(r"^\s*#\s*(?:if|ifdef|ifndef|elif)\b.*$", text, re.M):
            names = set(re.findall(r"\b([A-Z_][A-Z0-9_]*)\b", line)) - {"defined"}
            assert names and names <= allow, f"{f}: {line.strip()}"
            if f != "rx_config.h":
                assert names <= DIAGNOSTIC, f"{f}: {line.strip()} (knob defaults live in rx_config.h)"


def test_no_source_redefines_a_knob():
    allow = _allowlist()
    for f, text in _sources():
        if f == "rx_config.h":
            continue
        for k in allow:
            assert not re.search(rf"^\s*#\s*define\s+{k}\b", text, re.M), f"{f} defines {k}"
