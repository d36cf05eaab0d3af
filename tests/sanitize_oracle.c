/*
 * sanitize_oracle.c -- host-code sanitizer run of the CPU oracle (test
 * infrastructure; built and run by tests/test_sanitizers.py with
 * -fsanitize=address,undefined).  Exercises every oracle entry point on
 * ragged sizes, all G / R mixes, partial locks, `first` and copy flags, and
 * checks the fmaf restatements against the OpenBLAS replays bit for bit.
 * Exit status 0 = clean and equal.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../oracle/sma_oracle.h"

static int failures = 0;

static float *buf (size_t n, uint64_t seed, float sigma, const float *mean) {
	float *p = (float *) malloc (n * sizeof(float));
	cbo_fill_normal (p, n, seed, sigma, mean);
	return p;
}

static void same (const char *what, const float *a, const float *b, size_t n) {
	if (memcmp (a, b, n * sizeof(float)) != 0) {
		fprintf (stderr, "MISMATCH %s\n", what);
		failures++;
	}
}

static void sma_case (int G, int R, size_t n, float momentum, int first, int unlocked, int copy_id, int blas) {
	int size = G * R, i, g;
	float **z[2], **last[2], **s[2], **w[2];
	int *locked = (int *) calloc ((size_t) size, sizeof(int));
	int *copy[2];
	for (int v = 0; v < 2; ++v) {
		z[v] = (float **) calloc ((size_t) G, sizeof(float *));
		last[v] = (float **) calloc ((size_t) G, sizeof(float *));
		s[v] = (float **) calloc ((size_t) size, sizeof(float *));
		w[v] = (float **) calloc ((size_t) size, sizeof(float *));
		copy[v] = (int *) calloc ((size_t) size, sizeof(int));
		for (g = 0; g < G; ++g) {
			z[v][g] = buf (n, 1, 0.05f, NULL);
			last[v][g] = momentum > 0 ? buf (n, 2, 0.001f, NULL) : NULL;
		}
		for (i = 0; i < size; ++i) {
			s[v][i] = buf (n, 16 + 2 * i, 0.01f, z[v][i % G]);
			w[v][i] = buf (n, 17 + 2 * i, 0.001f, s[v][i]);
		}
		if (copy_id >= 0 && copy_id < size)
			copy[v][copy_id] = 1;
	}
	for (i = 0; i < size; ++i)
		locked[i] = (i != unlocked);
	float *scratch = (float *) malloc ((2 * (size_t) G * n + n) * sizeof(float));
	cbo_sma_fma (G, size, n, 0.1f, momentum, z[0], last[0], s[0], w[0], locked, copy[0], first, scratch);
	if (blas) {
		if (cbo_sma_blas (G, size, n, 0.1f, momentum, z[1], last[1], s[1], w[1], locked, copy[1], first, scratch) < 0) {
			fprintf (stderr, "BLAS replay unavailable\n");
			failures++;
		}
		for (g = 0; g < G; ++g) {
			same ("z", z[0][g], z[1][g], n);
			if (momentum > 0) same ("last", last[0][g], last[1][g], n);
		}
		for (i = 0; i < size; ++i) same ("w", w[0][i], w[1][i], n);
	}
	for (int v = 0; v < 2; ++v) {
		for (g = 0; g < G; ++g) { free (z[v][g]); free (last[v][g]); }
		for (i = 0; i < size; ++i) { free (s[v][i]); free (w[v][i]); }
		free (z[v]); free (last[v]); free (s[v]); free (w[v]); free (copy[v]);
	}
	free (locked);
	free (scratch);
}

static void step_cases (size_t n, int blas) {
	for (float mu = 0.0f; mu < 1.0f; mu += 0.9f) {
		for (int wdi = 0; wdi < 2; ++wdi) {
			float wd = wdi ? 5e-4f : 0.0f;
			float *w = buf (n, 100, 0.05f, NULL), *g = buf (n, 101, 0.01f, NULL), *l = buf (n, 102, 0.001f, NULL);
			float *z = buf (n, 103, 0.05f, NULL), *s = (float *) calloc (n, sizeof(float));
			float *w2 = malloc (n * 4), *g2 = malloc (n * 4), *l2 = malloc (n * 4), *z2 = malloc (n * 4), *s2 = calloc (n, 4);
			memcpy (w2, w, n * 4); memcpy (g2, g, n * 4); memcpy (l2, l, n * 4); memcpy (z2, z, n * 4);
			cbo_sma_optimise (n, -0.1f, mu, wd, w, g, mu > 0 ? l : NULL, s);
			cbo_default_task (n, -0.1f, mu, wd, w, g, mu > 0 ? l : NULL, z);
			cbo_ssgd_worker (n, -0.1f, wd, w, g, z);
			if (blas) {
				cbo_sma_optimise_blas (n, -0.1f, mu, wd, w2, g2, mu > 0 ? l2 : NULL, s2);
				cbo_default_task_blas (n, -0.1f, mu, wd, w2, g2, mu > 0 ? l2 : NULL, z2);
				cbo_ssgd_worker_blas (n, -0.1f, wd, w2, g2, z2);
				same ("optimise/default/ssgd w", w, w2, n);
				same ("g", g, g2, n);
				same ("z", z, z2, n);
				same ("s", s, s2, n);
			}
			free (w); free (g); free (l); free (z); free (s);
			free (w2); free (g2); free (l2); free (z2); free (s2);
		}
	}
}

int main (int argc, char **argv) {
	/* argv[1]: the OpenBLAS shared object to replay on (oracle.openblas_path()) */
	int blas = cbo_blas_open (argc > 1 ? argv[1] : NULL) == 0;
	if (! blas)
		fprintf (stderr, "note: no OpenBLAS found, fma restatement only\n");
	const size_t sizes[] = { 1, 3, 4099, 65537 };
	const int gs[] = { 1, 2, 4 }, rs[] = { 1, 3, 8 };
	for (int a = 0; a < 4; ++a)
		for (int b = 0; b < 3; ++b)
			for (int c = 0; c < 3; ++c) {
				sma_case (gs[b], rs[c], sizes[a], 0.9f, 0, -1, -1, blas);
				sma_case (gs[b], rs[c], sizes[a], 0.0f, 1, 0, gs[b] * rs[c] - 1, blas);
			}
	for (int a = 0; a < 4; ++a)
		step_cases (sizes[a], blas);
	/* BN averaging: 2 devices x 3 layers, one layer not updated on device 1 */
	{
		int G = 2, L = 3, elements[3] = { 5, 64, 1 }, updated[6] = { 1, 1, 1, 1, 0, 1 };
		float *mean[6], *var[6];
		for (int k = 0; k < G * L; ++k) {
			mean[k] = buf ((size_t) elements[k % L], 200 + k, 1.0f, NULL);
			var[k] = buf ((size_t) elements[k % L], 300 + k, 1.0f, NULL);
		}
		cbo_bn_average (G, L, elements, mean, var, updated);
		for (int k = 0; k < G * L; ++k) { free (mean[k]); free (var[k]); }
	}
	/* DEFAULT barrier */
	{
		size_t n = 777;
		float *z = buf (n, 400, 0.05f, NULL), *w[3];
		int locked[3] = { 1, 0, 1 };
		for (int i = 0; i < 3; ++i) w[i] = buf (n, 401 + i, 0.05f, NULL);
		cbo_default_sync (3, n, z, w, locked, 1);
		same ("default sync", w[2], z, n);
		for (int i = 0; i < 3; ++i) free (w[i]);
		free (z);
	}
	printf ("sanitize_oracle: %s (%s)\n", failures ? "FAILED" : "ok", blas ? cbo_blas_name () : "no BLAS");
	return failures ? 1 : 0;
}
