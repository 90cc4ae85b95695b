"""Copy integration/gpu_search.py (below its docstring) into INTEGRATION.md section 2."""
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
doc = (ROOT / "INTEGRATION.md").read_text()
body = (ROOT / "integration" / "gpu_search.py").read_text().split('"""\n', 1)[1]
head = "```python\n# src/xspect/models/gpu_search.py"
a = doc.index(head)
a = doc.index("\n", a) + 1
b = doc.index("```\n", a)
(ROOT / "INTEGRATION.md").write_text(doc[:a] + body + doc[b:])
