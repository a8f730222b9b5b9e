"""CPU oracle (test infrastructure only). See oracle/pst_oracle.c."""
