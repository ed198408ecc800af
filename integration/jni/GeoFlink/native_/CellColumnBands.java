/*
 * CellColumnBands -- the cell-column partitioner of the multi-GPU kNN (INTEGRATION.md §3,
 * DESIGN.md §7): a window's points are sharded over the GPUs of a node by bands of grid columns,
 * each band owned by one subtask = one GPU.  NOT COMPILED here (no JDK in the build image).
 *
 * Flink routes a keyed record to subtask KeyGroupRangeAssignment.assignKeyToParallelOperator(
 * key, maxParallelism, parallelism), a hash -- so the key of band b is chosen as the smallest
 * Integer that Flink sends to subtask b, and keyBy(new CellColumnBands(...)) delivers band b to
 * subtask b (its rank).  The job must fix maxParallelism (env.setMaxParallelism(M)) and the
 * operator's parallelism to nranks, and pass the same M here.
 *
 * Band of a point: its cell column (int) floor((x - minX) / cellLength) (HelperClass.java:109,
 * UniformGrid(int n, ...) cell length, UniformGrid.java:74-85), clamped to the grid (an
 * out-of-grid point goes to the edge band: the kNN cell filter rejects it on every rank anyway),
 * equal column ranges per band.  A heartbeat marker (marker(b)) is keyed to band b directly.
 */
package GeoFlink.native_;

import GeoFlink.spatialObjects.Point;
import org.apache.flink.api.java.functions.KeySelector;
import org.apache.flink.runtime.state.KeyGroupRangeAssignment;

public final class CellColumnBands implements KeySelector<Point, Integer> {
  /** objID prefix of the heartbeat markers (NaN coordinates; dropped by HipShardedKnnFunction) */
  public static final String MARKER = "\u0000gf-band-";

  private final int n, nranks;
  private final double minX, cellLength;
  private final int[] keyOfBand;

  public CellColumnBands(double[] gridArgs, int nranks, int maxParallelism) {
    this.n = (int) gridArgs[0];
    this.minX = gridArgs[1];
    this.cellLength = (gridArgs[2] - gridArgs[1]) / n;
    this.nranks = nranks;
    this.keyOfBand = new int[nranks];
    for (int b = 0; b < nranks; b++) {
      int key = 0;
      while (KeyGroupRangeAssignment.assignKeyToParallelOperator(key, maxParallelism, nranks) != b) key++;
      keyOfBand[b] = key;
    }
  }

  /** the band (= rank) owning a point's cell column */
  public int band(Point p) {
    if (p.objID != null && p.objID.startsWith(MARKER)) return Integer.parseInt(p.objID.substring(MARKER.length()));
    int c = (int) Math.floor((p.point.getX() - minX) / cellLength);
    c = c < 0 ? 0 : (c >= n ? n - 1 : c);
    return (int) ((long) c * nranks / n);
  }

  @Override
  public Integer getKey(Point p) { return keyOfBand[band(p)]; }

  /** a heartbeat point for band b: every band fires every window, so every rank makes the
   *  window's collective (a processing-time window fires per key only when the key has points) */
  public static Point marker(int band) {
    return new Point(MARKER + band, Double.NaN, Double.NaN, 0L);
  }

  public static boolean isMarker(Point p) { return p.objID != null && p.objID.startsWith(MARKER); }
}
