"""TEST INFRASTRUCTURE ONLY -- the CPU oracle of the X-ray render path.

Importable only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
leg.  The product (simpleraytracing_amd) never imports it.
"""
