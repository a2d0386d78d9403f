"""CPU oracle -- TEST INFRASTRUCTURE ONLY (see rbx_oracle.c header).  Never imported by redisson_amd/."""
