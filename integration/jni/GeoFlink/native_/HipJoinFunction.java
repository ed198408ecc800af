/*
 * HipJoinFunction -- the window body that replaces PointPointJoinQuery.windowBased
 * (PointPointJoinQuery.java:124-183): the query stream replicated to its neighbouring cells
 * (JoinQuery.getReplicatedPointQueryStream, JoinQuery.java:73-90), the cell-keyed window join and
 * the distance filter, as one device join per window.  NOT COMPILED here (no JDK in the build
 * image); see INTEGRATION.md and tests/test_shim_native.py (test_java_call_sequences).
 *
 * The reference:
 *   ordinary.join(replicatedQuery).where(gridID).equalTo(gridID)
 *       .window(SlidingProcessingTimeWindows.of(size, slide))
 *       .apply((p, q) -> approximate || distance(p, q) <= r ? (p, q) : (null, null))   // :148-175
 *       .filter(f1 != null)                                                            // :177-182
 * becomes
 *   ordinary.coGroup(query).where(p -> 0).equalTo(q -> 0)
 *       .window(SlidingProcessingTimeWindows.of(size, slide))
 *       .apply(new HipJoinFunction(uGridArgs, qGridArgs, r, approximate, device));
 * A constant key hands each window's two sides over whole; the replication, the key match and
 * the distance test are the device join (gf_join_pp: each (p, q) once, as the reference's
 * one-replica-per-cell join produces it).  Output: Tuple2(p, q) of the window's own Point
 * instances, ordered by (ordinary, query) window position.
 */
package GeoFlink.native_;

import GeoFlink.spatialObjects.Point;
import org.apache.flink.api.common.functions.RichCoGroupFunction;
import org.apache.flink.api.java.tuple.Tuple2;
import org.apache.flink.configuration.Configuration;
import org.apache.flink.util.Collector;

import java.util.ArrayList;

public class HipJoinFunction extends RichCoGroupFunction<Point, Point, Tuple2<Point, Point>> {

  private final double[] uGridArgs, qGridArgs;
  private final double radius;
  private final boolean approximate;
  private final int device;

  private transient long ctx;
  private transient HipColumns ocols, qcols;
  private transient ArrayList<Point> ordinary, query;

  public HipJoinFunction(double[] uGridArgs, double[] qGridArgs, double radius, boolean approximate, int device) {
    this.uGridArgs = uGridArgs.clone();
    this.qGridArgs = qGridArgs.clone();
    this.radius = radius;
    this.approximate = approximate;
    this.device = device;
  }

  @Override
  public void open(Configuration parameters) {
    ctx = GeoFlinkHip.ctxCreate(device);
    ocols = new HipColumns(false);
    qcols = new HipColumns(false);
    ordinary = new ArrayList<>();
    query = new ArrayList<>();
  }

  @Override
  public void close() {
    if (ctx != 0) GeoFlinkHip.ctxDestroy(ctx);
    ctx = 0;
  }

  @Override
  public void coGroup(Iterable<Point> ordinaryIn, Iterable<Point> queryIn, Collector<Tuple2<Point, Point>> out) {
    final int no = HipColumns.list(ordinaryIn, ordinary).size();
    final int nq = HipColumns.list(queryIn, query).size();
    if (no == 0 || nq == 0) return;
    ocols.fill(ctx, ordinary);
    qcols.fill(ctx, query);
    // pairs (ordinary index, query index) flattened; the context's pair buffer is sized from the
    // previous window and grown once when a window has more pairs
    final long[] pairs = GeoFlinkHip.joinWindow(ctx, uGridArgs, qGridArgs, ocols.x, ocols.y, no, qcols.x, qcols.y, nq,
                                                radius, approximate);
    for (int i = 0; i < pairs.length; i += 2)
      out.collect(Tuple2.of(ordinary.get((int) pairs[i]), query.get((int) pairs[i + 1])));
  }
}
