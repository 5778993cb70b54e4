# Top-level build: the product library and the (test-only) oracle.
all:
	$(MAKE) -C distributed-grep_amd
	$(MAKE) -C oracle

clean:
	$(MAKE) -C distributed-grep_amd clean
	$(MAKE) -C oracle clean

.PHONY: all clean
