// ORACLE TEST INFRASTRUCTURE — never part of the product path.
//
// Function-level harness around the UNMODIFIED reference translation unit
// (/root/reference/tsp.cpp, pulled in by the preprocessor at build time; no
// reference source is copied into this repository).  Built only in the
// survey container by oracle/Makefile into oracle/_ref/ (git-ignored), at -O0
// exactly like the reference's own Makefile (Makefile:3 has no -O flag), so
// that glibc pow() is really called (tsp.cpp -> assignment2.h:196).
//
// It exposes the reference's own functions so that fixtures can be generated:
//   gen   n B X Y      cities of distributeCities (tsp.cpp:373-403), %a exact
//   solve n B X Y      tsp() (tsp.cpp:405-509) on every generated block
//   solvefile FILE     tsp() on blocks read from FILE (for tie-heavy inputs)
//   dist  n B X Y      computeDistanceMatrix (assignment2.h:184-200)
//   fold  n B X Y      sequential mergeBlocks fold (tsp.cpp:202-269, 348-352)
//   time  n B X Y      wall time of tsp() per block (CPU baseline)
//   timeone n B X Y i  wall time of tsp() on block i only
// Output lines start with a tag so the generator's own printf
// ("%i blocks in X %i in Y", tsp.cpp:377) can be skipped by the reader.
#include <map>
#include <chrono>
#define main ref_main
#include "tsp.cpp"
#undef main

static void print_solution(const char *tag, int idx, const BlockSolution &s)
{
    printf("%s %d %a %.17g %zu", tag, idx, s.cost, s.cost, s.path.size());
    for (const City &c : s.path)
        printf(" %d", c.id);
    printf("\n");
}

static vector<vector<City>> generate(int n, int B, int X, int Y)
{
    srand(0);
    vector<int> dims = getBlocksPerDim(B);
    return distributeCities(n, dims[0], dims[1], X, Y);
}

static vector<vector<City>> read_blocks(const char *path)
{
    // Format: "B <count>" opens a block, then "<id> <x> <y>" lines (x,y as %a or decimal).
    vector<vector<City>> blocks;
    FILE *f = fopen(path, "r");
    if (!f)
    {
        perror(path);
        exit(2);
    }
    char tag[8];
    while (fscanf(f, "%7s", tag) == 1)
    {
        if (tag[0] == 'B')
        {
            int cnt;
            if (fscanf(f, "%d", &cnt) != 1)
                break;
            vector<City> blk;
            for (int i = 0; i < cnt; i++)
            {
                City c;
                char xs[64], ys[64];
                if (fscanf(f, "%d %63s %63s", &c.id, xs, ys) != 3)
                    exit(3);
                c.x = strtod(xs, nullptr);
                c.y = strtod(ys, nullptr);
                blk.push_back(c);
            }
            blocks.push_back(blk);
        }
    }
    fclose(f);
    return blocks;
}

int main(int argc, char **argv)
{
    if (argc < 3)
    {
        fprintf(stderr, "usage: ref_harness gen|solve|dist|fold|time n B X Y | timeone n B X Y i | solvefile FILE\n");
        return 1;
    }
    int only = -1;
    if (string(argv[1]) == "timeone" && argc == 7)
    {
        only = atoi(argv[6]);
        argc = 6;
    }
    procNum = 0;
    string cmd = argv[1];
    vector<vector<City>> blocks;
    if (cmd == "solvefile")
        blocks = read_blocks(argv[2]);
    else
    {
        if (argc != 6)
            return 1;
        blocks = generate(atoi(argv[2]), atoi(argv[3]), atoi(argv[4]), atoi(argv[5]));
    }

    if (cmd == "gen")
    {
        for (size_t b = 0; b < blocks.size(); b++)
            for (const City &c : blocks[b])
                printf("C %zu %d %a %a\n", b, c.id, c.x, c.y);
    }
    else if (cmd == "solve" || cmd == "solvefile")
    {
        for (size_t b = 0; b < blocks.size(); b++)
            print_solution("S", (int)b, tsp(blocks[b]));
    }
    else if (cmd == "dist")
    {
        for (size_t b = 0; b < blocks.size(); b++)
        {
            double **d = computeDistanceMatrix(blocks[b]);
            for (size_t i = 0; i < blocks[b].size(); i++)
                for (size_t j = 0; j < blocks[b].size(); j++)
                    printf("D %zu %zu %zu %a\n", b, i, j, d[i][j]);
        }
    }
    else if (cmd == "fold")
    {
        vector<BlockSolution> sols;
        for (size_t b = 0; b < blocks.size(); b++)
            sols.push_back(tsp(blocks[b]));
        BlockSolution acc = sols[0];
        print_solution("F", 0, acc);
        for (size_t b = 1; b < sols.size(); b++)
        {
            acc = mergeBlocks(acc, sols[b]);
            print_solution("F", (int)b, acc);
        }
    }
    else if (cmd == "time" || cmd == "timeone")
    {
        for (size_t b = 0; b < blocks.size(); b++)
        {
            if (only >= 0 && (int)b != only)
                continue;
            auto t0 = std::chrono::steady_clock::now();
            BlockSolution s = tsp(blocks[b]);
            auto t1 = std::chrono::steady_clock::now();
            printf("T %zu %.6f %a\n", b, std::chrono::duration<double>(t1 - t0).count(), s.cost);
        }
    }
    else
        return 1;
    return 0;
}
