// oracle_main.cpp -- TEST INFRASTRUCTURE ONLY: `oracle_photonmap src.scn out.png [-FLAGS]`,
// the CPU restatement behind the reference's CLI (photonmap.cpp:442-499).
extern "C" int oracle_main(int argc, char **argv);
int main(int argc, char **argv) { return oracle_main(argc, argv); }
