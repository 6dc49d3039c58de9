"""CPU: build the STOI stage-stamp analysis library (libcse_stamps.so beside
libcse.so; never the product build)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as g  # noqa: E402

g.build(out=os.path.join(g.PKG, "libcse_stamps.so"), defines=["CSE_STOI_STAMPS"])
print("built libcse_stamps.so")
