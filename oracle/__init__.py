"""Test-only oracles (see oracle/xcodec_oracle.c and oracle/ref_driver.cc)."""
