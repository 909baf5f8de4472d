# Construction-site dataset: schedule management initializer (reference
# datasets/construction/scripts/schedule-management/content/initializer/scheduleModel.groovy).

sb = schedule_builder
sb.persist(sb.new_simple_schedule("every-thirty-seconds", "Every thirty seconds", 30 * 1000))
sb.persist(sb.new_simple_schedule("every-minute", "Every minute", 60 * 1000))
sb.persist(sb.new_simple_schedule("every-ten-minutes", "Every 10 minutes", 10 * 60 * 1000))
sb.persist(sb.new_cron_schedule("on-the-half-hour", "On the half hour", "0,30 * * * *"))
sb.persist(sb.new_cron_schedule("every-hour", "On the hour", "0 * * * *"))
