"""Test-only oracle (CPU restatement of the reference forward). See ref_cpu.py header."""
