"""The native policies.yml reader (yaml.cpp, kw_yaml_to_json) against PyYAML's safe_load on every
policies file in the repo, the reference's YAML test inputs (config.rs:507-730, via
tests/golden/reference_cases.json), its policies.yml.example, and block-scalar / flow / quoting
samples. Samples stay inside the YAML 1.1 / 1.2 common ground: PyYAML resolves YAML 1.1 (`1e3` a
string, `0o17` a string, `017` octal) where serde_yaml, which the reference uses, follows 1.2
(`1e3` the float 1000.0); the native reader follows serde_yaml there (checked separately below)."""
import glob
import json
import os

import pytest
import yaml

import kwgpu as K
from helpers import ROOT, golden

SAMPLES = {
    "folded_blank_lines": "a: >\n  one\n  two\n\n  three\n\n\n  four\nb: 1\n",
    "folded_more_indented": "a: >\n  one\n    indented\n  two\n  three\n",
    "folded_strip": "a: >-\n  x\n\n  y\n\n",
    "folded_keep": "a: >+\n  x\n  y\n\n\nb: 2\n",
    "folded_keep_at_end": "a: >+\n  x\n\n",
    "literal": "a: |\n  line1\n\n  line3\n    deep\nb: |-\n  q\n",
    "literal_keep_at_end": "a: |+\n  x\n\n",
    "leading_blank": "a: >\n\n  x\n  y\n",
    "flow": "a: {x: 1, y: [1, 2, 'q'], z: \"s\"}\nb: [a, b,\n  c]\n",
    "quoting": "a: 'it''s'\nb: \"tab\\tend\"\nc: \"\\u00e9\"\nd: 'x: y'\n",
    "comments": "# c\na: 1 # trailing\nb:\n  - x # c\n  - y\n",
    "nested": "p:\n  settings:\n    list:\n    - a\n    - b: 1\n      c: [2]\n    empty:\n",
    "scalars": "a: true\nb: False\nc: ~\nd: 1.5\ne: -3\ng: .5\nh: 12345678901234567890123\ni: '007'\nj: registry://ghcr.io/x:v1\n",
    "plain_continued": "a: this is\n  continued\nb: x\n",
    "document_markers": "---\na: 1\n...\n",
}


def _docs():
    out = [(k, v) for k, v in SAMPLES.items()]
    for f in sorted(glob.glob(os.path.join(ROOT, "configs", "*.yml"))):
        out.append((os.path.basename(f), open(f).read()))
    out.append(("policies.yml.example", open(os.path.join(ROOT, "tests", "golden", "reference_data",
                                                         "policies.yml.example")).read()))
    cfg = golden("reference_cases.json")["config"]
    out.append(("read_policies_file", cfg["read_policies_file"]["yaml"]))
    for c in cfg["settings_conversion"]:
        out.append((c["ref"], c["yaml"]))
    return out


@pytest.mark.parametrize("name,text", _docs(), ids=lambda x: x if isinstance(x, str) and len(x) < 40 else None)
def test_native_yaml_equals_safe_load(name, text):
    assert K.yaml_to_json(text) == yaml.safe_load(text), name


@pytest.mark.parametrize("text", ["key: a: b\n", "k:\n  - x: y: z\n", "a: b:\n"])
def test_mapping_value_inside_plain_scalar_is_an_error(text):
    """`key: a: b` is not YAML (libyaml: "mapping values are not allowed in this context"); serde_yaml
    refuses it, so a policies.yml holding it does not load."""
    with pytest.raises(ValueError, match="mapping values"):
        K.yaml_to_json(text)
    with pytest.raises(yaml.YAMLError):
        yaml.safe_load(text)


def test_yaml_12_resolution_and_big_integers():
    """Where YAML 1.2 (serde_yaml) and 1.1 (PyYAML) part: exponent floats are numbers; integers past
    i64 keep their exact digits (no clamping)."""
    assert K.yaml_to_json("f: 1e3\ng: -2.5E-1\n") == {"f": 1000.0, "g": -0.25}
    assert K.yaml_to_json("h: 99999999999999999999\nk: -99999999999999999999\n") == {
        "h": 99999999999999999999, "k": -99999999999999999999}
    assert json.dumps(K.yaml_to_json("n: 9223372036854775807\n")) == '{"n": 9223372036854775807}'
