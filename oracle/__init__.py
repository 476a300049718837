"""TEST INFRASTRUCTURE ONLY -- parity checker for smallz4_amd (see smallz4_oracle.c)."""
