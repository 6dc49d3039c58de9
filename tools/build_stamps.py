"""CPU: build the stage-stamp analysis library (libcse_stamps.so beside
libcse.so; never the product build): STOI (CSE_STOI_STAMPS,
tools/stoi_stages.py) and enhance (CSE_ENH_STAMPS, tools/enhance_stages.py)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as g  # noqa: E402

g.build(out=os.path.join(g.PKG, "libcse_stamps.so"), defines=["CSE_STOI_STAMPS", "CSE_ENH_STAMPS"])
print("built libcse_stamps.so")
