/*
 * ShardedKnnPartial -- one rank's part of a window's merged kNN result (HipShardedKnnFunction):
 * the merged list's length m, and the entries whose Points this rank's band holds, each with its
 * rank in the merged (dist, objID) order.  ShardedKnnAssembler joins the nranks parts of a window.
 * NOT COMPILED here (no JDK in the build image).
 */
package GeoFlink.native_;

import GeoFlink.spatialObjects.Point;

import java.io.Serializable;
import java.util.ArrayList;

public class ShardedKnnPartial implements Serializable {
  public long windowStart, windowEnd;
  public int nranks, rank, m;
  public ArrayList<Integer> position = new ArrayList<>();
  public ArrayList<Point> points = new ArrayList<>();
  public ArrayList<Double> dist = new ArrayList<>();

  public ShardedKnnPartial() {}  // POJO

  public ShardedKnnPartial(long windowStart, long windowEnd, int nranks, int rank, int m) {
    this.windowStart = windowStart;
    this.windowEnd = windowEnd;
    this.nranks = nranks;
    this.rank = rank;
    this.m = m;
  }

  void add(int pos, Point p, double d) {
    position.add(pos);
    points.add(p);
    dist.add(d);
  }
}
