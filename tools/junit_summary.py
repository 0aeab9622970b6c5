"""Summarise a pytest junit report (tools/gpu.sh `tests` step) as one line per test + totals.
usage: python tools/junit_summary.py <junit.xml> [<pytest log>] > profiles/<round>/gpu_tests_summary.txt"""
import sys
import xml.etree.ElementTree as ET

root = ET.parse(sys.argv[1]).getroot()
suite = root if root.tag == "testsuite" else root.find("testsuite")
rows = []
for tc in suite.iter("testcase"):
    outcome = "PASSED"
    for tag in ("failure", "error", "skipped"):
        if tc.find(tag) is not None:
            outcome = tag.upper()
    rows.append((tc.get("classname", ""), tc.get("name", ""), float(tc.get("time", 0)), outcome))
print(f"# {suite.get('tests')} tests, {suite.get('failures')} failures, {suite.get('errors')} errors, "
      f"{suite.get('skipped')} skipped, {float(suite.get('time', 0)):.1f} s (junit report of the driver's command)")
for cls, name, t, outcome in rows:
    print(f"{cls.replace('.', '/')}.py::{name} {outcome} {t:.2f}s")
if len(sys.argv) > 2:
    lines = open(sys.argv[2]).read().strip().splitlines()
    print("# pytest: " + lines[-1] if lines else "# pytest: (empty log)")
