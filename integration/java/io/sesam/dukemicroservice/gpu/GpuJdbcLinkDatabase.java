package io.sesam.dukemicroservice.gpu;

import java.sql.Connection;
import java.sql.DriverManager;
import java.sql.PreparedStatement;
import java.sql.ResultSet;
import java.sql.SQLException;
import java.sql.Statement;
import java.sql.Timestamp;
import java.util.ArrayList;
import java.util.HashMap;
import java.util.HashSet;
import java.util.LinkedHashMap;
import java.util.List;
import java.util.Map;
import java.util.Properties;
import java.util.Set;

import no.priv.garshol.duke.Link;
import no.priv.garshol.duke.LinkKind;
import no.priv.garshol.duke.LinkStatus;
import no.priv.garshol.duke.links.JDBCLinkDatabase;

/**
 * The H2 link database (the default link-database-type, App.java:567-570, 597-602) with the
 * batch's links written in bulk -- OPT-IN (App.createLinkDatabase constructs this instead of
 * JDBCLinkDatabase when DUKEHIP_H2_BULK=true; INTEGRATION.md §3).
 *
 * Stock Duke writes the table per callback: LinkDatabaseMatchListener, per query record,
 * retracts the record's stored INFERRED links it did not produce again and asserts its new
 * ones, one statement each, and reads the table once per record (getAllLinksFor).  Here
 * GpuProcessor opens a listener window around each batch (its writes are dropped, as with
 * GpuLinkDatabase) and hands the batch's match arrays to applyBatch, which
 *   1. reads the stored links touching the batch's records in one SELECT (the IDs through a
 *      temporary table; an ASSERTED link is kept as [Duke 1.2, recalled] assertLink keeps it,
 *      Link.overrides),
 *   2. replays the listener's per-record rules in memory, in batch order (a later record sees
 *      what an earlier one wrote), and
 *   3. writes the final row of every touched link with one PreparedStatement batch (MERGE),
 *      committed once per deduplicate.
 * The final table equals the per-callback stream's (dukehip/jdbc_links.py is the Python
 * mirror, tests/test_jdbc_links.py checks it against that stream).
 *
 * PARITY UNPINNED against Duke: JDBCLinkDatabase is in the absent Duke 1.2 jar; its table
 * layout below is recalled ([Duke 1.2, recalled] links(id1, id2, kind, status, perhaps,
 * timestamp), key (id1, id2)), and so are the LinkKind / LinkStatus ids it stores.
 */
public class GpuJdbcLinkDatabase extends JDBCLinkDatabase {
    // [Duke 1.2 JDBCLinkDatabase, recalled]
    static final String TABLE = "links";
    static final String MERGE = "merge into " + TABLE
        + " (id1, id2, kind, status, perhaps, timestamp) key (id1, id2) values (?, ?, ?, ?, ?, ?)";

    private final String dburi;
    private final Properties props;
    private Connection conn;
    private boolean listenerWindow;   // GpuProcessor is inside a batch: listener writes dropped
    private int statements;           // SQL statements of the last batch

    public GpuJdbcLinkDatabase(String driverklass, String dburi, String dbtype, Properties props) {
        super(driverklass, dburi, dbtype, props);
        this.dburi = dburi;
        this.props = props == null ? new Properties() : props;
    }

    /**
     * GpuProcessor, around a batch's batchReady .. batchDone.  Opening the window commits the
     * superclass connection's pending writes first -- the routes' retractions of deleted
     * records' links (App.java:994-999) go through it before deduplicate runs, and with
     * auto-commit off they would stay uncommitted across the window: this class's own
     * connection would not see them in applyBatch's SELECT, and its MERGE of a link they
     * touched would wait on their row locks (tests/test_jdbc_links.py,
     * test_retraction_between_batches_two_connections, is the sqlite3 mirror).  Inside the
     * window the superclass connection writes nothing.
     */
    void setListenerWindow(boolean open) {
        if (open && !listenerWindow) super.commit();
        listenerWindow = open;
    }

    int lastBatchStatements() { return statements; }

    @Override
    public void assertLink(Link link) {
        if (listenerWindow) return;   // applyBatch writes the batch's links and retractions
        super.assertLink(link);       // the routes' own writes (deleted records, App.java:994-999)
    }

    @Override
    public void commit() {
        if (listenerWindow) return;   // batchDone's commit: applyBatch committed already
        super.commit();
    }

    private Connection connection() throws SQLException {
        if (conn == null) {
            conn = DriverManager.getConnection(dburi, props);   // H2 embedded: same process, same db
            conn.setAutoCommit(false);
        }
        return conn;
    }

    private static String[] key(String a, String b) {
        return a.compareTo(b) <= 0 ? new String[] {a, b} : new String[] {b, a};   // Link(id1, id2)
    }

    /**
     * One batch's match list: query record i (ID queryIds[i]) has entries first[i] ..
     * first[i+1]-1 (candidate ID, probability, DukeHip.KIND_MATCH / KIND_MAYBE), in batch order.
     * Returns the links written.
     */
    public int applyBatch(String[] queryIds, long[] first, String[] candidateIds, double[] prob,
                          byte[] kind, long timestamp) {
        final int inferred = LinkStatus.INFERRED.getId(), retracted = LinkStatus.RETRACTED.getId();
        try {
            Connection c = connection();
            statements = 0;
            final int asserted = LinkStatus.ASSERTED.getId();
            // 1. the stored links of the batch's records (every status: an ASSERTED one stays)
            Map<String, Object[]> state = new HashMap<>();   // "id1\0id2" -> {id1, id2, kind, status, perhaps, ts}
            Map<String, Set<String>> byId = new HashMap<>();
            try (Statement st = c.createStatement()) {
                st.execute("create local temporary table if not exists dk_batch_ids (id varchar(200) primary key)");
                st.execute("delete from dk_batch_ids");
                statements += 2;
            }
            try (PreparedStatement ins = c.prepareStatement("merge into dk_batch_ids (id) key (id) values (?)")) {
                Set<String> seen = new HashSet<>();
                for (String q : queryIds) if (seen.add(q)) { ins.setString(1, q); ins.addBatch(); }
                ins.executeBatch();
                statements += 1;
            }
            try (PreparedStatement sel = c.prepareStatement(
                     "select id1, id2, kind, status, perhaps, timestamp from " + TABLE + " where "
                     + "id1 in (select id from dk_batch_ids) or id2 in (select id from dk_batch_ids)")) {
                try (ResultSet rs = sel.executeQuery()) {
                    while (rs.next()) {
                        Object[] row = {rs.getString(1), rs.getString(2), rs.getInt(3), rs.getInt(4),
                                        rs.getDouble(5), rs.getTimestamp(6).getTime()};
                        String k = row[0] + "\0" + row[1];
                        state.put(k, row);
                        byId.computeIfAbsent((String) row[0], x -> new HashSet<>()).add(k);
                        byId.computeIfAbsent((String) row[1], x -> new HashSet<>()).add(k);
                    }
                }
                statements += 1;
            }
            // 2. LinkDatabaseMatchListener's per-record rules, in batch order
            Map<String, Object[]> fin = new LinkedHashMap<>();
            for (int i = 0; i < queryIds.length; i++) {
                String q = queryIds[i];
                Map<String, Object[]> cur = new LinkedHashMap<>();
                for (long e = first[i]; e < first[i + 1]; e++) {
                    String[] k2 = key(q, candidateIds[(int) e]);
                    int lk = kind[(int) e] == DukeHip.KIND_MATCH ? LinkKind.SAME.getId() : LinkKind.MAYBE.getId();
                    cur.put(k2[0] + "\0" + k2[1], new Object[] {k2[0], k2[1], lk, inferred, prob[(int) e], timestamp});
                }
                Set<String> mine = byId.get(q);
                if (mine != null) {
                    for (String k : new ArrayList<>(mine)) {
                        Object[] row = state.get(k);
                        if (cur.containsKey(k) || (Integer) row[3] != inferred) continue;
                        Object[] r = {row[0], row[1], row[2], retracted, row[4], timestamp};
                        state.put(k, r);
                        fin.put(k, r);
                    }
                }
                for (Map.Entry<String, Object[]> en : cur.entrySet()) {
                    Object[] r = en.getValue();
                    Object[] old = state.get(en.getKey());
                    if (old != null && (Integer) old[3] == asserted) continue;   // Link.overrides
                    state.put(en.getKey(), r);
                    fin.put(en.getKey(), r);
                    byId.computeIfAbsent((String) r[0], x -> new HashSet<>()).add(en.getKey());
                    byId.computeIfAbsent((String) r[1], x -> new HashSet<>()).add(en.getKey());
                }
            }
            // 3. the final row of every touched link, one batch, one commit
            try (PreparedStatement m = c.prepareStatement(MERGE)) {
                for (Object[] r : fin.values()) {
                    m.setString(1, (String) r[0]);
                    m.setString(2, (String) r[1]);
                    m.setInt(3, (Integer) r[2]);
                    m.setInt(4, (Integer) r[3]);
                    m.setDouble(5, (Double) r[4]);
                    m.setTimestamp(6, new Timestamp((Long) r[5]));
                    m.addBatch();
                }
                m.executeBatch();
                statements += 1;
            }
            c.commit();
            statements += 1;
            return fin.size();
        } catch (SQLException ex) {
            throw new RuntimeException("bulk link write failed", ex);
        }
    }

    @Override
    public void close() {
        try {
            if (conn != null) conn.close();
        } catch (SQLException ignored) {
            // the superclass's connection is closed below either way
        }
        super.close();
    }
}
