"""Extract the golden (payload, expected SQL) vectors from the reference's own plan test.

Source: /root/reference/query-api/src/test/scala/com/cardinal/queryapi/utils/ASTUtilsBaseExprTest.scala
(testTagApiShouldNotDoASelectStar 71-74, testQueryApiPayloadWithExtract 205-215,
testGroupByOnExtractedField 274-288).  Only the string literals (data) are kept, in
tests/golden/ref_sql_cases.json; this script runs in the build container only (the reference does not
exist on the GPU box).
"""
import json
import os
import re
import sys

SRC = "/root/reference/query-api/src/test/scala/com/cardinal/queryapi/utils/ASTUtilsBaseExprTest.scala"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "ref_sql_cases.json")


def strip_margin(s: str) -> str:
    return "\n".join(re.sub(r"^\s*\|", "", line) for line in s.split("\n"))


def main():
    text = open(SRC).read()
    blocks = re.findall(r'"""(.*?)"""(?!")', text, flags=re.S)
    payloads = [strip_margin(b) for b in blocks if "baseExpressions" in b]
    sqls = [strip_margin(b).strip() for b in blocks if b.lstrip("|").lstrip().startswith("SELECT") or
            b.lstrip().startswith("|SELECT")]
    ts_uses = re.findall(r"val ts: Long = (\d+)L", text)
    cases = [
        {"name": "tag_query", "payload": json.loads(payloads[0]), "expr": "A", "kind": "tag_filter_sql",
         "start": 1, "end": 1, "expected": sqls[0], "cite": "ASTUtilsBaseExprTest.scala:71-74"},
        {"name": "chart_with_extract", "payload": json.loads(payloads[1]), "expr": "A", "kind": "chart_sql",
         "start": int(ts_uses[0]), "end": int(ts_uses[0]), "step": 10000, "expected": sqls[1],
         "cite": "ASTUtilsBaseExprTest.scala:205-211"},
        {"name": "groupby_extracted", "payload": json.loads(payloads[2]), "expr": "a", "kind": "chart_sql",
         "start": int(ts_uses[1]), "end": int(ts_uses[1]), "step": 10000, "expected": sqls[3],
         "cite": "ASTUtilsBaseExprTest.scala:274-288"},
    ]
    with open(OUT, "w") as f:
        json.dump(cases, f, indent=1)
    print(f"wrote {len(cases)} cases to {OUT}", file=sys.stderr)


if __name__ == "__main__":
    main()
