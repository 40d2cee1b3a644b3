// One reference test (tests/<name>.cpp of the reference, compiled unmodified
// with -Dmain=<name>_main as its CMakeLists.txt:55-61 does) as an executable
// of its own, so that a test that aborts (sync_word_test overflows its heap
// buffer) leaves the others' results standing.  Built by
// oracle/Makefile `harness`; TEST_MAIN names the test's renamed main.
int TEST_MAIN();
int main() { return TEST_MAIN(); }
