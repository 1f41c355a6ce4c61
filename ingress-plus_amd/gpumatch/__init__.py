"""gpumatch -- host side of the MI355X batched request-matching engine.

* ``confgen``  -- Configurator restatement: Ingress / VirtualServer -> nginx text (fixtures)
* ``records``  -- packed ``gm_req`` records + synthetic workloads C1..C5
* ``sigs``     -- WAF signature sets
* ``blob``     -- GMB1 generation blobs (what Manager.Reload hands to the engine)
* ``engine``   -- ctypes binding of libgpumatch.so (the C-ABI in include/gpumatch.h)
* ``manager``  -- nginx.Manager-shaped wrapper (Python mirror of the Go cgo wrapper)
"""
