# Repository-level targets.  The product library and the oracle are built by
# __graft_entry__.build() (allpathslg_amd/csrc/Makefile, oracle/Makefile).
#   make sanitize   host code + CPU restatement under ASan/UBSan and TSan
#                   (tests/sanitize)
sanitize:
	$(MAKE) -C tests/sanitize all

.PHONY: sanitize
